-- Lua 5.4 pieces the round-5 interpreter lacked (string.pack family, load's env / _ENV, to-be-closed
-- variables, __gc finalizers and collectgarbage, the debug library): each block asserts the values
-- a luaL_openlibs state gives (splinter_cli_cmd_lua.c:395).
local function eq(a, b, msg)
  if a ~= b then error((msg or "check") .. ": got " .. tostring(a) .. " want " .. tostring(b), 2) end
end

-- string.pack / unpack / packsize
eq(string.pack("<i4", 100), "\100\0\0\0", "pack i4")
eq(string.pack(">i2", 1), "\0\1", "pack big i2")
eq(string.unpack("<i2", "\255\255"), -1, "unpack i2")
eq(select(2, string.unpack("<i2", "\255\255")), 3, "unpack next pos")
eq(string.unpack("<I2", "\255\255"), 65535, "unpack I2")
eq(string.pack(">I3", 0x010203), "\1\2\3", "pack I3")
eq(string.packsize("i4i8"), 12, "packsize no align")
eq(string.packsize("!i4i8"), 16, "packsize native align")
eq(string.packsize("!4 i1 i4"), 8, "packsize !4")
eq(string.packsize("!8 i1 Xi8"), 8, "packsize X")
eq(string.pack("i1 x i1", 1, 2), "\1\0\2", "pad byte")
eq(string.pack("z", "hi"), "hi\0", "pack z")
local zs, zn = string.unpack("z", "hi\0rest")
eq(zs, "hi", "unpack z")
eq(zn, 4, "unpack z pos")
eq(string.pack("s1", "abc"), "\3abc", "pack s1")
eq(string.unpack("s1", "\3abcdef"), "abc", "unpack s1")
eq(string.unpack("d", string.pack("d", 1.5)), 1.5, "double")
eq(string.unpack("f", string.pack("f", 0.5)), 0.5, "float")
eq(string.unpack("<j", string.pack("<j", -2)), -2, "j")
eq(string.unpack("<i16", string.pack("<i16", -3)), -3, "i16")
eq(string.unpack(">i3", string.pack(">i3", -70000)), -70000, "i3 sign")
local a1, a2, a3 = string.unpack("<i2 i2", string.pack("<i2 i2", 7, -7))
eq(a1 + a2, 0, "two values")
eq(a3, 5, "next after two")
eq(string.unpack("<i2", "xx\1\0", 3), 1, "init position")
local ok, err = pcall(string.pack, "i1", 200)
eq(ok, false, "overflow")
eq(err:find("overflow") ~= nil, true, "overflow message")
ok, err = pcall(string.unpack, "i4", "ab")
eq(ok, false, "short data")
ok, err = pcall(string.packsize, "s")
eq(ok, false, "packsize variable")

-- load(chunk, name, mode, env) and _ENV
local env = {x = 5}
eq(load("return x", "c", "t", env)(), 5, "load env read")
load("y = 7", "c", "t", env)()
eq(env.y, 7, "load env write")
eq(y, nil, "load env keeps globals")
eq(load("return tostring(1)", "c", "t", setmetatable({}, {__index = _G}))(), "1", "env __index")
local function scoped()
  local _ENV = {v = 9}
  return v
end
eq(scoped(), 9, "local _ENV")
eq(_ENV, _G, "_ENV is _G")
local f2, msg = load("return 1", "c", "b")
eq(f2, nil, "mode b refuses text")

-- to-be-closed variables
local log = {}
local function closer(tag)
  return setmetatable({}, {__close = function(_, e) log[#log + 1] = tag .. (e and (":" .. tostring(e)) or "") end})
end
do
  local a <close> = closer("a")
  local b <close> = closer("b")
  local n <close> = nil
  local k <const> = 5
  eq(k, 5, "const")
end
eq(table.concat(log, ","), "b,a", "close order")
log = {}
local function ret1()
  local c <close> = closer("r")
  return 1
end
eq(ret1(), 1, "return value")
eq(log[1], "r", "closed on return")
log = {}
for i = 1, 3 do
  local c <close> = closer("i" .. i)
  if i == 2 then break end
end
eq(table.concat(log, ","), "i1,i2", "closed on break")
log = {}
ok, err = pcall(function()
  local c <close> = closer("e")
  error("boom", 0)
end)
eq(ok, false, "error propagates")
eq(log[1], "e:boom", "close gets the error")
ok, err = pcall(load, "local x <close> = 1")
local fnc = load("local x <close> = 1")
ok, err = pcall(fnc)
eq(ok, false, "non-closable")
eq(err:find("non%-closable") ~= nil, true, "non-closable message")
eq(load("local a <foo> = 1"), nil, "unknown attribute")

-- __gc and collectgarbage
local gc_log = {}
do
  local t = setmetatable({}, {__gc = function(o) gc_log[#gc_log + 1] = "t" end})
end
collectgarbage()
eq(#gc_log, 1, "finalized once unreachable")
local held = setmetatable({}, {__gc = function() gc_log[#gc_log + 1] = "held" end})
collectgarbage("collect")
eq(#gc_log, 1, "reachable not finalized")
eq(type(collectgarbage("count")), "number", "count")
eq(collectgarbage("isrunning"), true, "isrunning")
keep_until_close = setmetatable({}, {__gc = function() print("FINALIZED AT CLOSE") end})

-- debug
eq(debug.traceback("x"):sub(1, 18), "x\nstack traceback:", "traceback")
eq(debug.traceback({}) ~= nil, true, "traceback non-string passthrough")
eq(debug.getinfo(print).what, "C", "getinfo C")
eq(debug.getinfo(function(p, q) end).nparams, 2, "getinfo nparams")
local mt = {__metatable = "locked"}
local o = setmetatable({}, mt)
eq(getmetatable(o), "locked", "protected")
eq(debug.getmetatable(o), mt, "debug.getmetatable raw")
debug.setmetatable(o, nil)
eq(getmetatable(o), nil, "debug.setmetatable")
debug.sethook()
eq(debug.gethook(), nil, "gethook")
eq(type(debug.getregistry()), "table", "registry")

print("ALL OK")
