"""tensor_filter framework=lua (reference ext/nnstreamer/tensor_filter/tensor_filter_lua.cc,
tests/nnstreamer_filter_lua/unittest_filter_lua.cc patterns: script and file modes,
two-tensor passthrough + constant output, invalid script / TensorsInfo, out-of-range
tensor and element indices, every element type) on the built-in Lua 5.1 subset
interpreter (csrc/filter/lua_vm.cc)."""
import textwrap
import time

import numpy as np
import pytest

TWO_TENSORS = textwrap.dedent("""
    inputTensorsInfo = {
      num = 2,
      dim = {{3, 100, 100, 1}, {3, 24, 24, 1},},
      type = {'uint8', 'uint8',}
    }
    outputTensorsInfo = {
      num = 2,
      dim = {{3, 100, 100, 1}, {2, 1, 1, 1},},
      type = {'uint8', 'float32',}
    }
    function nnstreamer_invoke()
      input = input_tensor(1)
      output = output_tensor(1)
      for i=1,3*100*100*1 do
        output[i] = input[i]
      end
      input = input_tensor(2)
      output = output_tensor(2)
      for i=1,2 do
        output[i] = i * 11
      end
    end
""")


def _inputs():
    rng = np.random.default_rng(0)
    return [rng.integers(0, 256, (100, 100, 3), dtype=np.uint8), rng.integers(0, 256, (24, 24, 3), dtype=np.uint8)]


def _check_two(ys, xs):
    np.testing.assert_array_equal(np.asarray(ys[0]).reshape(-1), xs[0].reshape(-1))
    np.testing.assert_array_equal(np.asarray(ys[1]).reshape(-1), np.array([11, 22], np.float32))


def test_script_mode(nns):
    with nns.Single(TWO_TENSORS, framework="lua") as s:
        assert [t.getDims()[:4] for t in s.input_info] == [[3, 100, 100, 1], [3, 24, 24, 1]]
        assert [t.getDims()[:4] for t in s.output_info] == [[3, 100, 100, 1], [2, 1, 1, 1]]
        xs = _inputs()
        _check_two(s.invoke(*xs), xs)


def test_file_mode_and_pipeline(nns, tmp_path):
    f = tmp_path / "passthrough.lua"
    f.write_text(TWO_TENSORS)
    xs = _inputs()
    with nns.Single(str(f), framework="lua") as s:
        _check_two(s.invoke(*xs), xs)
    # auto framework from the .lua extension, inside a pipeline
    caps = "other/tensors,num_tensors=2,format=static,dimensions=3:100:100:1.3:24:24:1,types=uint8.uint8,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter framework=auto model={f} ! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda b: got.append([b.memory(0).numpy("uint8").copy(),
                                                                  b.memory(1).numpy("float32").copy()]))
    p.set_state("playing")
    for i in range(3):
        p.get_by_name("src").push_buffer(list(xs), pts=i)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    assert len(got) == 3
    for ys in got:
        _check_two(ys, xs)


def test_missing_dims_default_to_one_and_types(nns):
    script = textwrap.dedent("""
        inputTensorsInfo = { num = 1, dim = {{4}}, type = {'int16'} }
        outputTensorsInfo = { num = 4, dim = {{4}, {4}, {4}, {2, 2}}, type = {'float64', 'uint8', 'int32', 'float16'} }
        function nnstreamer_invoke()
          local x = input_tensor(1)
          local a, b, c, d = output_tensor(1), output_tensor(2), output_tensor(3), output_tensor(4)
          for i = 1, #x do
            a[i] = x[i] / 4       -- float64 keeps the fraction
            b[i] = x[i] + 256     -- uint8 wraps
            c[i] = -x[i] * 1000
            d[i] = x[i] * 0.5
          end
        end
    """)
    with nns.Single(script, framework="lua") as s:
        assert s.input_info[0].getDims()[:4] == [4, 1, 1, 1]
        assert s.output_info[3].getDims()[:4] == [2, 2, 1, 1]
        x = np.array([1, 2, 3, 7], np.int16)
        a, b, c, d = s.invoke(x)
        np.testing.assert_array_equal(np.asarray(a).view(np.float64).reshape(-1), x / 4)
        np.testing.assert_array_equal(np.asarray(b).view(np.uint8).reshape(-1), (x.astype(np.int64) + 256) % 256)
        np.testing.assert_array_equal(np.asarray(c).view(np.int32).reshape(-1), -x.astype(np.int32) * 1000)
        np.testing.assert_array_equal(np.asarray(d).view(np.float16).reshape(-1), (x * 0.5).astype(np.float16))


@pytest.mark.parametrize("script", [
    "this is not lua",
    "inputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }\n"
    "outputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }\n",  # no nnstreamer_invoke
    "inputTensorsInfo = { num = 17, dim = {{1}}, type = {'uint8'} }\n"
    "outputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }\nfunction nnstreamer_invoke() end",
    "inputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint7'} }\n"
    "outputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }\nfunction nnstreamer_invoke() end",
    "inputTensorsInfo = { num = 1, dim = {{'a'}}, type = {'uint8'} }\n"
    "outputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }\nfunction nnstreamer_invoke() end",
    "inputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }\nfunction nnstreamer_invoke() end",
    "error('load-time failure')",
])
def test_invalid_script_fails_to_open(nns, script):
    with pytest.raises(Exception):
        nns.Single(script, framework="lua")


_IO = "inputTensorsInfo = { num = 1, dim = {{4}}, type = {'float32'} }\n" \
      "outputTensorsInfo = { num = 1, dim = {{4}}, type = {'float32'} }\n"


@pytest.mark.parametrize("body", [
    "output_tensor(2)[1] = 0",          # the script declares one output
    "output_tensor(17)[1] = 0",         # beyond the tensor limit
    "output_tensor(0)[1] = 0",
    "output_tensor(1)[5] = 0",          # element out of range
    "output_tensor(1)[0] = 0",
    "input_tensor(1)[1] = 0",           # inputs are read-only
    "output_tensor(1)[1] = {}",
    "local x = nil + 1",
    "while true do end",                # stopped by custom=max_steps
])
def test_invoke_errors(nns, body):
    script = _IO + f"function nnstreamer_invoke()\n  {body}\nend\n"
    with nns.Single(script, framework="lua", custom="max_steps:100000") as s:
        with pytest.raises(Exception):
            s.invoke(np.zeros(4, np.float32))


def test_handle_kept_past_invoke_is_refused(nns):
    script = _IO + textwrap.dedent("""
        kept = nil
        function nnstreamer_invoke()
          if kept then kept[1] = 1 end   -- the handle from the previous frame
          kept = output_tensor(1)
        end
    """)
    with nns.Single(script, framework="lua") as s:
        s.invoke(np.zeros(4, np.float32))
        with pytest.raises(Exception):
            s.invoke(np.zeros(4, np.float32))


def test_language_subset(nns):
    """Closures, varargs, multiple returns, tables, generic for, string and
    math libraries, pcall, method calls, long strings and comments: every
    result lands in one float64 output."""
    script = textwrap.dedent(r"""
        --[[ a long
             comment ]]
        inputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }
        outputTensorsInfo = { num = 1, dim = {{16}}, type = {'float64'} }
        local function counter()
          local n = 0
          return function(k) n = n + (k or 1); return n end
        end
        local function sum(...)
          local s = 0
          for _, v in ipairs({...}) do s = s + v end
          return s, select('#', ...)
        end
        local function fib(n) if n < 2 then return n end return fib(n - 1) + fib(n - 2) end
        local Acc = {}
        function Acc.new(v) return { v = v, add = function(self, d) self.v = self.v + d; return self end } end
        function nnstreamer_invoke()
          local o = output_tensor(1)
          local c = counter(); c(); c(5)
          o[1] = c()                                   -- 7
          local s, n = sum(1, 2, 3, 4)
          o[2] = s; o[3] = n                           -- 10, 4
          o[4] = fib(15)                               -- 610
          local t = { 10, 20, 30, x = 5, ["y z"] = 6 }
          local keys = 0
          for k, v in pairs(t) do keys = keys + 1 end
          o[5] = keys + #t                             -- 5 + 3
          o[6] = #string.format("%05.1f|%d|%s", 3.14159, 42, "ab")   -- "003.1|42|ab" = 11
          o[7] = tonumber("0x1F") + tonumber("  12  ")  -- 43
          local ok, err = pcall(function() error("boom") end)
          o[8] = (not ok and string.find(err, "boom")) and 1 or 0
          o[9] = Acc.new(1):add(2):add(3).v            -- 6
          o[10] = math.floor(7 / 2) + 7 % 3 + 2 ^ 3     -- 3 + 1 + 8
          local parts = {}
          for i = 10, 1, -3 do table.insert(parts, i) end
          o[11] = tonumber(table.concat(parts, ""))     -- 10741
          o[12] = #[[abc
        def]]                                          -- 7
          local r = 0
          repeat r = r + 1 until r >= 4
          while true do r = r + 1; if r > 6 then break end end
          o[13] = r                                    -- 7
          o[14] = ("Lua"):upper() == "LUA" and 1 or 0
          o[15] = (1 == 1.0 and "a" < "b" and not (nil or false)) and 1 or 0
          o[16] = -2 ^ 2                               -- -4 (power binds tighter)
        end
    """)
    with nns.Single(script, framework="lua") as s:
        (y,) = s.invoke(np.zeros(1, np.uint8))
        got = np.asarray(y).view(np.float64).reshape(-1).tolist()
    assert got == [7, 10, 4, 610, 8, 11, 43, 1, 6, 12, 10741, 7, 7, 1, 1, -4]


def test_reload_on_model_change(nns, tmp_path):
    """is-updatable: a new script replaces the running one between frames."""
    a, b = tmp_path / "a.lua", tmp_path / "b.lua"
    body = "function nnstreamer_invoke() output_tensor(1)[1] = input_tensor(1)[1] * {k} end\n"
    a.write_text(_IO + body.format(k=2))
    b.write_text(_IO + body.format(k=3))
    caps = "other/tensors,num_tensors=1,format=static,dimensions=4,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter name=f framework=lua model={a} "
                         "is-updatable=true ! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda b: got.append(float(b.memory(0).numpy("float32")[0])))
    p.set_state("playing")
    src = p.get_by_name("src")
    src.push_buffer(np.full(4, 5, np.float32), pts=0)
    t0 = time.time()
    while len(got) < 1 and time.time() - t0 < 10:
        time.sleep(0.01)
    p.get_by_name("f").set_property("model", str(b))
    src.push_buffer(np.full(4, 5, np.float32), pts=1)
    src.end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    assert got == [10.0, 15.0]


def test_closures_capture_per_iteration_and_through_levels(nns):
    """Lua 5.1 upvalue rules: each loop iteration's locals are fresh, closures
    share a captured variable, and an upvalue is reachable two functions up."""
    script = textwrap.dedent("""
        inputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }
        outputTensorsInfo = { num = 1, dim = {{8}}, type = {'float64'} }
        function nnstreamer_invoke()
          local o = output_tensor(1)
          local fs = {}
          for i = 1, 3 do fs[i] = function() return i * 10 end end
          o[1], o[2], o[3] = fs[1](), fs[2](), fs[3]()          -- 10 20 30
          local gs = {}
          local j = 0
          while j < 2 do j = j + 1; local k = j; gs[j] = function() return k end end
          o[4] = gs[1]() + 10 * gs[2]()                          -- 21
          local shared = 1
          local function inc() shared = shared + 1 end
          local function get() return shared end
          inc(); inc()
          o[5] = get()                                           -- 3
          local function outer()
            local v = 5
            return function() return function() v = v + 1; return v end end
          end
          local h = outer()()
          h()
          o[6] = h()                                             -- 7
          local x = 1
          do local x = x + 1; o[7] = x end                       -- 2 (inner x sees the outer)
          o[8] = x                                               -- 1
        end
    """)
    with nns.Single(script, framework="lua") as s:
        (y,) = s.invoke(np.zeros(1, np.uint8))
        got = np.asarray(y).view(np.float64).reshape(-1).tolist()
    assert got == [10, 20, 30, 21, 3, 7, 2, 1]


_REF_MODELS = "/root/reference/tests/test_models/models"


@pytest.mark.parametrize("name", ["passthrough.lua", "scaler.lua"])
def test_reference_model_scripts(nns, name):
    """The reference's own Lua test models (tests/test_models/models/*.lua) run
    unchanged; the scaler is a nearest-neighbour 640x480 -> 320x240 resize."""
    import os
    path = os.path.join(_REF_MODELS, name)
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    x = np.random.default_rng(3).integers(0, 256, (480, 640, 3), dtype=np.uint8)
    with nns.Single(path, framework="lua") as s:
        (y,) = s.invoke(x)
    y = np.asarray(y).reshape(-1)
    if name == "passthrough.lua":
        np.testing.assert_array_equal(y, x.reshape(-1))
    else:
        hs = np.floor(np.arange(240) * (480 / 240)).astype(int)
        ws = np.floor(np.arange(320) * (640 / 320)).astype(int)
        np.testing.assert_array_equal(y.reshape(240, 320, 3), x[hs][:, ws])


def test_metatables_patterns_and_libraries(nns):
    """Lua 5.1 features beyond the tensor scripts' core: metatables (OOP via
    __index, operators, __call, __tostring, __newindex), Lua patterns
    (find / match / gmatch / gsub with captures, sets, anchors, %b), table.sort
    and the os / math.random subset -- results land in a float64 output."""
    script = textwrap.dedent(r"""
        inputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }
        outputTensorsInfo = { num = 1, dim = {{20}}, type = {'float64'} }
        local Vec = {}
        Vec.__index = Vec
        function Vec.new(x, y) return setmetatable({x = x, y = y}, Vec) end
        function Vec:len2() return self.x * self.x + self.y * self.y end
        Vec.__add = function(a, b) return Vec.new(a.x + b.x, a.y + b.y) end
        Vec.__eq = function(a, b) return a.x == b.x and a.y == b.y end
        Vec.__lt = function(a, b) return a:len2() < b:len2() end
        Vec.__le = function(a, b) return a:len2() <= b:len2() end
        Vec.__unm = function(a) return Vec.new(-a.x, -a.y) end
        Vec.__tostring = function(a) return "(" .. a.x .. "," .. a.y .. ")" end
        Vec.__concat = function(a, b) return tostring(a) .. tostring(b) end
        Vec.__call = function(self, k) return self.x * k end
        function nnstreamer_invoke()
          local o = output_tensor(1)
          local v = Vec.new(1, 2) + Vec.new(3, 4)
          o[1] = v:len2()                                             -- 16 + 36 = 52
          o[2] = (Vec.new(1, 1) == Vec.new(1, 1)) and 1 or 0          -- 1
          o[3] = (Vec.new(1, 1) < Vec.new(2, 2)) and 1 or 0           -- 1
          o[4] = (-v).x                                                -- -4
          o[5] = #tostring(v)                                          -- "(4,6)" = 5
          o[6] = v(10)                                                 -- 40
          o[7] = #(Vec.new(1, 2) .. Vec.new(3, 4))                     -- "(1,2)(3,4)" = 10
          local log = {}
          local proxy = setmetatable({}, {__newindex = function(t, k, val) rawset(t, k, val * 2); log[#log + 1] = k end})
          proxy.a = 5
          o[8] = proxy.a + #log                                        -- 10 + 1
          local defaults = setmetatable({}, {__index = function(t, k) return #k end})
          o[9] = defaults.hello                                        -- 5
          local s, e, word = string.find("say hello world", "(%a+)", 5)
          o[10] = s * 100 + e                                          -- 5*100 + 9
          o[11] = tonumber(string.match("id=42;", "id=(%d+)"))         -- 42
          local sum = 0
          for n in string.gmatch("1, 22, 333", "%d+") do sum = sum + tonumber(n) end
          o[12] = sum                                                  -- 356
          local r, n = string.gsub("hello world", "(%w+)", "<%1>")
          o[13] = #r * 10 + n                                          -- "<hello> <world>" 15 -> 152
          local r2 = string.gsub("abc", "%w", {a = "1", b = false})   -- "1bc": false keeps the match
          local r3 = string.gsub(r2, "%a", function(c) return c == "c" and "3" or nil end)
          o[14] = (r3 == "1b3") and 1 or 0
          o[15] = (string.find("f(a(b)c)d", "%b()")) or -1             -- 2
          o[16] = (string.match("  trim me  ", "^%s*(.-)%s*$") == "trim me") and 1 or 0
          local t = {5, 3, 9, 1}
          table.sort(t)
          o[17] = t[1] * 1000 + t[2] * 100 + t[3] * 10 + t[4]          -- 1359
          table.sort(t, function(a, b) return a > b end)
          o[18] = t[1]                                                 -- 9
          math.randomseed(7)
          local a1 = math.random(1, 100)
          math.randomseed(7)
          o[19] = (a1 == math.random(1, 100) and a1 >= 1 and a1 <= 100) and 1 or 0
          o[20] = (os.clock() >= 0 and os.time() > 1e9 and #os.date("%Y") == 4) and 1 or 0
        end
    """)
    with nns.Single(script, framework="lua") as s:
        (y,) = s.invoke(np.zeros(1, np.uint8))
        got = np.asarray(y).view(np.float64).reshape(-1).tolist()
    assert got == [52, 1, 1, -4, 5, 40, 10, 11, 5, 509, 42, 356, 152, 1, 2, 1, 1359, 9, 1, 1]


@pytest.mark.parametrize("expr,want", [
    ('select(2, string.gsub("hello", "", "-"))', 6),                  # empty pattern matches 6 times
    ('#(string.gsub("hello", "", "-"))', 11),                         # "-h-e-l-l-o-"
    ('select(2, string.gsub("aaa", "^a", "b"))', 1),                  # anchored: one substitution
    ('string.find("THE (quick) fox", "%((%a+)%)")', 5),
    ('select(3, string.find("hello", "()ll()"))', 3),                 # position captures
    ('select(2, string.find("abcabc", "(abc)%1"))', 6),               # back-reference
    ('string.find("THE quick", "%f[%a]%a+", 4)', 5),                  # frontier
    ('#string.match("key = value", "(%w+)%s*=%s*(%w+)")', 3),
    ('string.find("a.b", ".", 1, true) + string.find("a.b", "%.")', 4),
    ('select("#", string.match("2024-01-15", "(%d+)-(%d+)-(%d+)"))', 3),
    ('tonumber(string.format("%.2f", 3.14159)) * 100', 314),
    ('string.byte("AB", 1, 2) + select(2, string.byte("AB", 1, 2))', 131),
    ('#string.rep("ab", 3) + #string.reverse("xyz")', 9),
    ('(string.match("[[nested]]", "%[(%b[])%]")) == "[nested]" and 1 or 0', 1),
])
def test_lua_pattern_semantics(nns, expr, want):
    script = ("inputTensorsInfo = { num = 1, dim = {{1}}, type = {'uint8'} }\n"
              "outputTensorsInfo = { num = 1, dim = {{1}}, type = {'float64'} }\n"
              f"function nnstreamer_invoke() output_tensor(1)[1] = {expr} end\n")
    with nns.Single(script, framework="lua") as s:
        (y,) = s.invoke(np.zeros(1, np.uint8))
    assert np.asarray(y).view(np.float64)[0] == want


def test_runaway_recursion_and_nesting_fail_cleanly(nns):
    """Unbounded recursion through pcall ends at the interpreter's depth cap
    (each pcall level sees the error) instead of overflowing the C++ stack, and
    a script nested deeper than the parser allows fails to load."""
    script = _IO + textwrap.dedent("""
        function nnstreamer_invoke()
          local depth = 0
          local function f(n) depth = math.max(depth, n); pcall(f, n + 1) end
          f(1)
          output_tensor(1)[1] = depth
        end
    """)
    with nns.Single(script, framework="lua") as s:
        (y,) = s.invoke(np.zeros(4, np.float32))
        assert 100 <= np.asarray(y).view(np.float32)[0] <= 200
        (y,) = s.invoke(np.zeros(4, np.float32))  # the depth counter was restored
        assert 100 <= np.asarray(y).view(np.float32)[0] <= 200
    deep = _IO + "x = " + "(" * 5000 + "1" + ")" * 5000 + "\nfunction nnstreamer_invoke() end\n"
    with pytest.raises(Exception):
        nns.Single(deep, framework="lua")
