-- Lua 5.4 standard library and goto, as the reference gets them from luaL_openlibs
-- (splinter_cli_cmd_lua.c:395): each block asserts its expected values.
local function eq(a, b, msg)
  if a ~= b then error((msg or "check") .. ": got " .. tostring(a) .. " want " .. tostring(b), 2) end
end

-- table.sort / table.move / table.pack
local t = {5, 2, 9, 1, 7, 3}
table.sort(t)
eq(table.concat(t, ","), "1,2,3,5,7,9", "sort")
table.sort(t, function(a, b) return a > b end)
eq(table.concat(t, ","), "9,7,5,3,2,1", "sort desc")
local w = {"pear", "apple", "fig"}
table.sort(w)
eq(table.concat(w, " "), "apple fig pear", "sort strings")
local big = {}
for i = 1, 500 do big[i] = (i * 7919) % 1009 end
table.sort(big)
for i = 2, 500 do assert(big[i - 1] <= big[i], "sorted big") end
local m = table.move({1, 2, 3, 4, 5}, 2, 4, 1)
eq(table.concat(m, ","), "2,3,4,4,5", "move in place")
local dst = table.move({1, 2, 3}, 1, 3, 2, {})
eq(dst[2] .. dst[3] .. dst[4], "123", "move to other")
local pk = table.pack(1, nil, 3)
eq(pk.n, 3, "pack.n")

-- goto
local out = {}
for i = 1, 6 do
  if i % 3 == 0 then goto continue end
  out[#out + 1] = i
  ::continue::
end
eq(table.concat(out, ","), "1,2,4,5", "goto continue")

-- math.type
eq(math.type(1), "integer"); eq(math.type(1.5), "float"); eq(math.type("1"), nil)
eq(math.ult(1, -1), true, "ult")

-- string.format %q
eq(string.format("%q", 'a "b"\n'), '"a \\"b\\"\\\n"', "%q")

-- os.date / os.time
local tt = os.date("*t", 86400 * 365)
eq(type(tt.year), "number"); eq(tt.month >= 1 and tt.month <= 12, true)
eq(os.date("!%Y-%m-%d", 0), "1970-01-01", "date utc")
eq(os.time({year = 2020, month = 1, day = 2, hour = 0}) - os.time({year = 2020, month = 1, day = 1, hour = 0}), 86400)

-- io: open / write / read / lines / seek / close; os.rename / os.remove
local path = os.tmpname()
local f = assert(io.open(path, "w"))
f:write("line one\n", "line two\n", 42, "\n")
f:close()
eq(io.type(f), "closed file")
f = assert(io.open(path, "r"))
eq(io.type(f), "file")
eq(f:read("l"), "line one")
eq(f:read("L"), "line two\n")
eq(f:read("n"), 42)
f:seek("set", 0)
eq(#f:read("a"), 21, "read all")
f:close()
local n = 0
for line in io.lines(path) do n = n + 1 end
eq(n, 3, "io.lines")
local p2 = path .. ".moved"
assert(os.rename(path, p2))
eq(io.open(path, "r"), nil, "renamed away")
assert(os.remove(p2))
local ok, err = os.remove(p2)
eq(ok, nil); eq(type(err), "string")
io.write("io.write works", "\n")

-- load / loadstring / dofile
local fn = load("local a, b = ... return a * b")
eq(fn(6, 7), 42, "load")
eq(loadstring("return 1 + 1")(), 2, "loadstring")
local bad, msg = load("return +")
eq(bad, nil); eq(type(msg), "string")
local parts = {"return ", "'pie", "ce'"}
local i = 0
eq(load(function() i = i + 1 return parts[i] end)(), "piece", "load reader")
local lp = os.tmpname()
local g = io.open(lp, "w"); g:write("return ...  or 'dofile ok'"); g:close()
eq(dofile(lp), "dofile ok", "dofile")
os.remove(lp)

-- utf8
eq(utf8.char(72, 228, 8364, 128512), "H\xC3\xA4\xE2\x82\xAC\xF0\x9F\x98\x80", "utf8.char")
local s = "h\xC3\xA4\xE2\x82\xACx"
eq(utf8.len(s), 4, "utf8.len")
eq(select(2, utf8.codepoint(s, 1, -1)), 228, "codepoint")
eq(utf8.offset(s, 3), 4, "offset")
local cps = {}
for p, c in utf8.codes(s) do cps[#cps + 1] = p .. ":" .. c end
eq(table.concat(cps, " "), "1:104 2:228 4:8364 7:120", "codes")
eq(utf8.len("\xFF"), nil, "invalid utf8")

print("ALL OK")
