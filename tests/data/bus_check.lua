-- splinter module smoke check for the `lua` verb (mirrors what the reference's
-- CLI regression runs through `splinterctl lua`): args, get/set, math on BIGUINT.
local bus = require("splinter")
print("script: " .. arg[0] .. " args=" .. #arg)
local v = bus.get("test_key") or "missing"
print("test_key=" .. v)
assert(bus.set("lua_text", "1, 2, 3"))
assert(bus.set("lua_counter", 41))
assert(bus.math("lua_counter", "inc", 1))
assert(bus.get("lua_counter") == 42, "counter")
assert(bus.set_tandem("lua_t", {"a", "b", "c"}))
local t = bus.get_tandem("lua_t")
assert(#t == 3 and t[3] == "c", "tandem")
assert(bus.label("lua_text", 0x10))
assert(bus.bump("lua_text"))
local ok, err = pcall(bus.math, "lua_text", "inc", 1)
assert(not ok and err:find("BIGUINT"), "math on text must fail")
local vec = {}
for i = 1, 768 do vec[i] = (i % 7) / 7 end
assert(bus.set_embedding("lua_text", vec))
local back = bus.get_embedding("lua_text")
assert(back and math.abs(back[8] - 1 / 7) < 1e-6, "embedding")
print(string.format("ok %d", bus.get("lua_counter")))
