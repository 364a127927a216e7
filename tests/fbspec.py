"""A FlatBuffers reader and writer written from the binary format's rules, for
the nnstreamer.flatbuf.Tensors schema (reference
ext/nnstreamer/include/nnstreamer.fbs:1-65), independent of csrc/serial:

* the buffer starts with a uoffset (u32) to the root table;
* a table starts with an soffset (i32): its vtable is at table - soffset (before
  or after the table); the vtable is [u16 vtable bytes][u16 table bytes][u16
  field offsets...], 0 or a missing entry = the field's default;
* string / vector / sub-table fields hold a uoffset relative to the field's own
  position (so they point forward); a vector is [u32 count][elements], a string
  [u32 length][bytes][NUL]; a struct (frame_rate: two int32) is inline.

No flatbuffers library is importable here: this pins the codec against the
format and the schema, not against flatc's particular layout.
"""
import struct

TYPE_DEFAULT = 10  # NNS_END


class Reader:
    def __init__(self, b):
        self.b = bytes(b)

    def u32(self, at):
        return struct.unpack_from("<I", self.b, at)[0]

    def i32(self, at):
        return struct.unpack_from("<i", self.b, at)[0]

    def field(self, t, fid):
        vt = t - self.i32(t)
        vsz = struct.unpack_from("<H", self.b, vt)[0]
        at = 4 + 2 * fid
        if at + 2 > vsz:
            return None
        o = struct.unpack_from("<H", self.b, vt + at)[0]
        return t + o if o else None

    def deref(self, at):
        return at + self.u32(at)

    def tensors(self):
        t = self.deref(0)
        f = self.field(t, 0)
        num = self.i32(f) if f else 0
        f = self.field(t, 1)
        fr = struct.unpack_from("<ii", self.b, f) if f else (0, 0)
        f = self.field(t, 3)
        fmt = self.i32(f) if f else 0
        out = []
        f = self.field(t, 2)
        if f:
            vec = self.deref(f)
            for i in range(self.u32(vec)):
                tt = self.deref(vec + 4 + 4 * i)
                g = self.field(tt, 0)
                name = ""
                if g:
                    s = self.deref(g)
                    name = self.b[s + 4:s + 4 + self.u32(s)].decode()
                g = self.field(tt, 1)
                typ = self.i32(g) if g else TYPE_DEFAULT
                g = self.field(tt, 2)
                dims = []
                if g:
                    v = self.deref(g)
                    dims = list(struct.unpack_from(f"<{self.u32(v)}I", self.b, v + 4))
                g = self.field(tt, 3)
                data = b""
                if g:
                    v = self.deref(g)
                    data = self.b[v + 4:v + 4 + self.u32(v)]
                out.append(dict(name=name, type=typ, dims=dims, data=data))
        return dict(num_tensor=num, fr=fr, format=fmt, tensor=out)


class Writer:
    """Front-to-back layout with knobs a reader must tolerate: vtables after
    their tables (negative soffset), one vtable shared by every Tensor table,
    inline fields in a non-schema order, and unknown trailing fields."""

    def __init__(self):
        self.b = bytearray()

    def pad(self, a):
        while len(self.b) % a:
            self.b.append(0)

    def put(self, fmt, *v):
        self.pad(struct.calcsize(fmt) if fmt[-1] in "iIHQq" else 1)
        at = len(self.b)
        self.b += struct.pack("<" + fmt, *v)
        return at

    def patch_uoff(self, field_at, target):
        struct.pack_into("<I", self.b, field_at, target - field_at)

    def build(self, tensors, fr=(30, 1), fmt=0, vtable_after=True, shared_vtable=True, extra_field=True):
        root = self.put("I", 0)
        # Tensors table, inline order: [soff][format][tensor uoff][fr.n][fr.d][num_tensor][unknown]
        self.pad(8)
        t = self.put("i", 0)
        f_fmt = self.put("i", fmt)
        f_vec = self.put("I", 0)
        f_fr = self.put("ii", *fr)
        f_num = self.put("i", len(tensors))
        f_x = self.put("i", 12345) if extra_field else None
        offs = [f_num - t, f_fr - t, f_vec - t, f_fmt - t] + ([f_x - t] if extra_field else [])
        tsize = len(self.b) - t
        if vtable_after:
            vt = self.put("H", 4 + 2 * len(offs))
            self.put("H", tsize)
            for o in offs:
                self.put("H", o)
        else:
            raise ValueError("only the vtable-after form is built here")
        struct.pack_into("<i", self.b, t, t - vt)
        self.patch_uoff(root, t)
        # vector of Tensor table offsets
        vec = self.put("I", len(tensors))
        self.patch_uoff(f_vec, vec)
        slots = [self.put("I", 0) for _ in tensors]
        shared = None
        for slot, ten in zip(slots, tensors):
            # Tensor inline order: [soff][data uoff][type][dims uoff][name uoff]
            self.pad(4)
            tt = self.put("i", 0)
            g_data = self.put("I", 0)
            g_type = self.put("i", ten["type"])
            g_dims = self.put("I", 0)
            g_name = self.put("I", 0)
            toffs = [g_name - tt, g_type - tt, g_dims - tt, g_data - tt]
            if shared is None or not shared_vtable:
                v = self.put("H", 4 + 2 * len(toffs))
                self.put("H", g_name + 4 - tt)
                for o in toffs:
                    self.put("H", o)
                shared = v
            struct.pack_into("<i", self.b, tt, tt - shared)
            self.patch_uoff(slot, tt)
            # children: data first, then dims, then the name
            dv = self.put("I", len(ten["data"]))
            self.b += ten["data"]
            self.patch_uoff(g_data, dv)
            mv = self.put("I", len(ten["dims"]))
            for d in ten["dims"]:
                self.put("I", d)
            self.patch_uoff(g_dims, mv)
            sv = self.put("I", len(ten["name"]))
            self.b += ten["name"].encode() + b"\0"
            self.patch_uoff(g_name, sv)
        self.pad(4)
        return bytes(self.b)
