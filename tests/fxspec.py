"""A FlexBuffers reader and writer written from the format's rules, for the map
tensordec-flexbuf.cc:120-160 builds ({num_tensors: UInt, rate_n / rate_d /
format: Int, tensor_<i>: [name: String, type: Int, dimension: typed UInt vector,
data: Blob]}), independent of csrc/serial:

* the last byte is the root slot's width, the one before it the root's packed
  type ((type << 2) | log2(child width)), the root slot precedes them;
* offset values (strings, blobs, keys, vectors, maps) are unsigned distances
  BACK from the slot that holds them; a vector is [size][elements][one packed
  type per element] with the size and elements at the child width, a typed
  vector has no type bytes, a string / blob is [size][bytes] (+ NUL), a key is
  NUL-terminated bytes, a map is [keys offset][keys width][size][values][types]
  with its keys a typed key vector in strcmp order.

The writer picks the narrowest width that holds every slot of a vector, as the
flexbuffers builder does (the reference decoder's output is byte-narrow for
small frames), where csrc/serial's encoder writes every slot 8 bytes wide.
No flatbuffers library is importable here.
"""
import struct

NULL, INT, UINT, FLOAT, KEY, STRING = 0, 1, 2, 3, 4, 5
MAP, VECTOR, VECTOR_INT, VECTOR_UINT, VECTOR_KEY, BLOB = 9, 10, 11, 12, 14, 25
_FMT = {1: "B", 2: "H", 4: "I", 8: "Q"}
_SFMT = {1: "b", 2: "h", 4: "i", 8: "q"}


def _code(w):
    return {1: 0, 2: 1, 4: 2, 8: 3}[w]


class Reader:
    def __init__(self, b):
        self.b = bytes(b)

    def uint(self, at, w):
        return struct.unpack_from("<" + _FMT[w], self.b, at)[0]

    def sint(self, at, w):
        return struct.unpack_from("<" + _SFMT[w], self.b, at)[0]

    def value(self, slot, pw, packed):
        t, cw = packed >> 2, 1 << (packed & 3)
        if t == INT:
            return self.sint(slot, pw)
        if t == UINT:
            return self.uint(slot, pw)
        target = slot - self.uint(slot, pw)
        if t in (STRING, BLOB):
            n = self.uint(target - cw, cw)
            raw = self.b[target:target + n]
            return raw.decode() if t == STRING else raw
        if t == KEY:
            return self.b[target:self.b.index(b"\0", target)].decode()
        if t in (VECTOR_INT, VECTOR_UINT):
            n = self.uint(target - cw, cw)
            rd = self.sint if t == VECTOR_INT else self.uint
            return [rd(target + i * cw, cw) for i in range(n)]
        if t == VECTOR:
            n = self.uint(target - cw, cw)
            return [self.value(target + i * cw, cw, self.b[target + n * cw + i]) for i in range(n)]
        if t == MAP:
            n = self.uint(target - cw, cw)
            kslot = target - 3 * cw
            keys_at = kslot - self.uint(kslot, cw)
            kw = self.uint(target - 2 * cw, cw)
            keys = [self.value(keys_at + i * kw, kw, KEY << 2) for i in range(n)]
            vals = [self.value(target + i * cw, cw, self.b[target + n * cw + i]) for i in range(n)]
            return dict(zip(keys, vals))
        raise ValueError(f"flexbuffers type {t} not in this schema")

    def root(self):
        rw = self.b[-1]
        return self.value(len(self.b) - 2 - rw, rw, self.b[-2])


def _uwidth(v):
    return 1 if v < 1 << 8 else 2 if v < 1 << 16 else 4 if v < 1 << 32 else 8


def _swidth(v):
    return 1 if -128 <= v < 128 else 2 if -32768 <= v < 32768 else 4 if -2 ** 31 <= v < 2 ** 31 else 8


class Writer:
    def __init__(self):
        self.b = bytearray()

    def align(self, w):
        while len(self.b) % w:
            self.b.append(0)

    def put(self, v, w, signed=False):
        self.b += struct.pack("<" + (_SFMT if signed else _FMT)[w], v)

    def sized(self, data, nul):
        w = _uwidth(len(data))
        self.align(w)
        self.put(len(data), w)
        at = len(self.b)
        self.b += data + (b"\0" if nul else b"")
        return at, w

    def typed_uint(self, vals):
        w = _uwidth(max(max(vals), len(vals)))
        self.align(w)
        self.put(len(vals), w)
        at = len(self.b)
        for v in vals:
            self.put(v, w)
        return at, w

    def build(self, tensors, rate=(30, 1), fmt=0):
        vals = {"num_tensors": ("u", len(tensors), UINT << 2), "rate_n": ("s", rate[0], INT << 2),
                "rate_d": ("s", rate[1], INT << 2), "format": ("s", fmt, INT << 2)}
        for i, t in enumerate(tensors):
            name, nw = self.sized(t["name"].encode(), True)
            dims, dw = self.typed_uint(t["dims"])
            data, bw = self.sized(t["data"], False)
            elems = [("o", name, STRING << 2 | _code(nw)), ("s", t["type"], INT << 2 | _code(_swidth(t["type"]))),
                     ("o", dims, VECTOR_UINT << 2 | _code(dw)), ("o", data, BLOB << 2 | _code(bw))]
            vec, vw = self._vec_with_types(elems)
            vals[f"tensor_{i}"] = ("o", vec, VECTOR << 2 | _code(vw))
        order = sorted(vals)  # strcmp order of the keys
        kpos = {}
        for k in order:
            kpos[k] = len(self.b)
            self.b += k.encode() + b"\0"
        keys, kw = self._typed_offsets([kpos[k] for k in order])
        elems = [vals[k] for k in order]
        m, mw = self._vec_with_types(elems, keys=(keys, kw))
        # root slot: the narrowest width that holds the distance back to the map
        rw = 1
        while True:
            at = (len(self.b) + rw - 1) // rw * rw
            if at - m < 1 << (8 * rw):
                break
            rw *= 2
        self.align(rw)
        self.put(len(self.b) - m, rw)
        self.b.append(MAP << 2 | _code(mw))
        self.b.append(rw)
        return bytes(self.b)

    def _typed_offsets(self, targets):
        for w in (1, 2, 4, 8):
            start = (len(self.b) + w - 1) // w * w
            pos = start + w
            if all(0 <= pos + i * w - t < 1 << (8 * w) for i, t in enumerate(targets)) and len(targets) < 1 << (8 * w):
                break
        self.align(w)
        self.put(len(targets), w)
        for i, t in enumerate(targets):
            self.put(len(self.b) - t, w)
        return pos, w

    def _vec_with_types(self, elems, keys=None):
        """[size][elements][types], narrowest width; a map (keys = (keys vector
        position, its width)) has [keys offset][keys width] before the size"""
        npre = 2 if keys else 0
        for w in (1, 2, 4, 8):
            start = (len(self.b) + w - 1) // w * w
            pos = start + (npre + 1) * w
            ok = len(elems) < 1 << (8 * w)
            if keys:
                ok = ok and 0 <= start - keys[0] < 1 << (8 * w) and keys[1] < 1 << (8 * w)
            for i, (k, v, _) in enumerate(elems):
                x = pos + i * w - v if k == "o" else v
                ok = ok and (_swidth(x) <= w if k == "s" else 0 <= x < 1 << (8 * w))
            if ok:
                break
        self.align(w)
        if keys:
            self.put(len(self.b) - keys[0], w)  # keys vector offset
            self.put(keys[1], w)                # keys width
        self.put(len(elems), w)
        assert len(self.b) == pos
        for k, v, _ in elems:
            self.put(len(self.b) - v if k == "o" else v, w, signed=(k == "s"))
        for _, _, packed in elems:
            self.b.append(packed)
        return pos, w
