-- Lua 5.4 semantics of string patterns and metatables in splinterctl's interpreter
-- (expected values are the reference liblua5.4 behaviour of each call)
local function eq(a, b, msg)
  if a ~= b then error((msg or "check") .. ": got " .. tostring(a) .. " want " .. tostring(b), 2) end
end

-- string.find
eq(string.find("hello world", "wor"), 7)
local s, e = string.find("hello world", "o w"); eq(s, 5); eq(e, 7)
s, e = string.find("hello", "l+"); eq(s, 3); eq(e, 4)
eq(string.find("a.b", ".", 1, true), 2)
eq(string.find("abc", "^b"), nil)
s, e = string.find("abc", "^a"); eq(s, 1); eq(e, 1)
local x1, x2, k, v = string.find("key=val", "(%w+)=(%w+)")
eq(x1, 1); eq(x2, 7); eq(k, "key"); eq(v, "val")

-- string.match
eq(string.match("hello 123 world", "%d+"), "123")
local k2, v2 = string.match("  name = value ", "(%w+)%s*=%s*(%w+)"); eq(k2, "name"); eq(v2, "value")
local p1, p2 = string.match("abc", "()b()"); eq(p1, 2); eq(p2, 3)
eq(string.match("2024-01-15", "(%d+)-(%d+)-(%d+)"), "2024")
eq(select(3, string.match("2024-01-15", "(%d+)-(%d+)-(%d+)")), "15")
eq(string.match("THE (quick) fox", "%((%a+)%)"), "quick")
eq(string.match("f(a(b)c)d", "%b()"), "(a(b)c)")
eq(string.match("hello", ".-l"), "hel")
eq(string.match("hello", ".*l"), "hell")
eq(string.match("aaa", "a-b"), nil)
eq(string.match("abab", "(ab)%1"), "ab")
eq(select(2, string.match("x = 'quoted'", "(['\"])(.-)%1")), "quoted")
eq(string.match("THE (quick) fox", "%f[%a]%a+"), "THE")
eq(string.match("[test]", "[]]"), "]")
eq(string.match("a-b", "[a-]+"), "a-")
eq(string.match("x9y", "[^%a]"), "9")
eq(string.match("hello", "^(h)(e)"), "h")
eq(string.match("end", "d$"), "d")
eq(string.match("x", "y?x"), "x")
eq(string.match("  trim  ", "^%s*(.-)%s*$"), "trim")
eq(string.match("abc123", "%a+"), "abc")
eq(string.match("abc123", "%A+"), "123")
eq(string.match("hello", "l", 4), "l")
eq(string.match("hello", "h", 2), nil)
eq(string.match("hello", "o", -1), "o")

-- string.gmatch
local words = {}
for w in string.gmatch("one two  three", "%a+") do words[#words + 1] = w end
eq(#words, 3); eq(words[3], "three")
local t = {}
for kk, vv in string.gmatch("a=1, b=2, c=3", "(%w+)=(%w+)") do t[kk] = tonumber(vv) end
eq(t.a, 1); eq(t.c, 3)
local cnt = 0
for _ in ("abc"):gmatch("") do cnt = cnt + 1 end
eq(cnt, 4)

-- string.gsub
eq(string.gsub("hello world", "o", "0"), "hell0 w0rld")
eq(select(2, string.gsub("hello world", "o", "0")), 2)
eq(string.gsub("hello world", "(%w+)", "<%1>"), "<hello> <world>")
eq(string.gsub("hello", "", "-"), "-h-e-l-l-o-")
eq(string.gsub("abc", "%w", "%0%0"), "aabbcc")
eq(string.gsub("hello world", "%w+", string.upper), "HELLO WORLD")
eq(string.gsub("$name is $age", "%$(%w+)", {name = "Bob", age = 42}), "Bob is 42")
eq(string.gsub("$name is $x", "%$(%w+)", {name = "Bob"}), "Bob is $x")
eq(string.gsub("hello world", "o", "0", 1), "hell0 world")
eq(string.gsub("aaa", "^a", "X"), "Xaa")
eq(string.gsub("one two", "(%w+) (%w+)", "%2 %1"), "two one")
eq(string.gsub("50%", "%%", " percent"), "50 percent")
assert(not pcall(string.find, "a", "[a"))
assert(not pcall(string.match, "a", "%"))
assert(not pcall(string.gsub, "a", "a", "%2"))

-- metatables
local V = {}
V.__index = V
V.__add = function(a, b) return setmetatable({x = a.x + b.x}, V) end
V.__eq = function(a, b) return a.x == b.x end
V.__lt = function(a, b) return a.x < b.x end
V.__le = function(a, b) return a.x <= b.x end
V.__tostring = function(o) return "V(" .. o.x .. ")" end
V.__len = function(o) return o.x end
V.__call = function(self, y) return self.x * y end
V.__concat = function(a, b) return tostring(a) .. "|" .. tostring(b) end
V.__unm = function(a) return setmetatable({x = -a.x}, V) end
function V.new(x) return setmetatable({x = x}, V) end
function V:double() return self.x * 2 end
local a, b = V.new(2), V.new(3)
eq((a + b).x, 5)
eq(a:double(), 4)
eq(tostring(a), "V(2)")
eq(a == V.new(2), true)
eq(a ~= b, true)
eq(a < b, true); eq(b <= a, false); eq(b > a, true); eq(a >= b, false)
eq(#b, 3)
eq(a(10), 20)
eq(a .. b, "V(2)|V(3)")
eq((-a).x, -2)
eq(getmetatable(a), V)

local log = {}
local proxy = setmetatable({}, {
  __index = function(_, key) return key .. "!" end,
  __newindex = function(tt, key, val) log[#log + 1] = key; rawset(tt, key, val) end})
eq(proxy.foo, "foo!")
proxy.bar = 1
eq(rawget(proxy, "bar"), 1); eq(log[1], "bar")
proxy.bar = 2
eq(#log, 1)

local Base = {greet = function() return "hi" end}
local Mid = setmetatable({}, {__index = Base})
local obj = setmetatable({}, {__index = Mid})
eq(obj.greet(), "hi")

local prot = setmetatable({}, {__metatable = "locked"})
eq(getmetatable(prot), "locked")
assert(not pcall(setmetatable, prot, {}))

local pp = setmetatable({}, {__pairs = function(tt)
  return function(_, kk) if not kk then return 1, "one" end end, tt, nil
end})
local seen
for _, vv in pairs(pp) do seen = vv end
eq(seen, "one")

eq(("%d-%d"):format(1, 2), "1-2")
eq(getmetatable("").__index, string)
print("ALL OK")
