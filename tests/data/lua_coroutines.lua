-- coroutine library semantics (Lua 5.4 reference behaviour)
local function eq(a, b, msg)
  if a ~= b then error((msg or "check") .. ": got " .. tostring(a) .. " want " .. tostring(b), 2) end
end

local co = coroutine.create(function(a, b)
  eq(coroutine.status(coroutine.running()), "running")
  local c = coroutine.yield(a + b)
  local d, e = coroutine.yield(c * 2)
  return d + e, "done"
end)
eq(type(co), "thread")
eq(coroutine.status(co), "suspended")
local ok, v = coroutine.resume(co, 1, 2); eq(ok, true); eq(v, 3)
ok, v = coroutine.resume(co, 10); eq(ok, true); eq(v, 20)
local ok2, s, tag = coroutine.resume(co, 4, 5); eq(ok2, true); eq(s, 9); eq(tag, "done")
eq(coroutine.status(co), "dead")
ok, v = coroutine.resume(co); eq(ok, false); eq(v, "cannot resume dead coroutine")

-- generator via wrap
local function range(n)
  return coroutine.wrap(function() for i = 1, n do coroutine.yield(i) end end)
end
local sum = 0
for i in range(5) do sum = sum + i end
eq(sum, 15)

-- errors inside a coroutine come back from resume; wrap re-raises them
local bad = coroutine.create(function() error("boom", 0) end)
ok, v = coroutine.resume(bad); eq(ok, false); eq(v, "boom")
local w = coroutine.wrap(function() error({code = 7}) end)
local pok, perr = pcall(w); eq(pok, false); eq(perr.code, 7)

-- yield across pcall and nested Lua calls
local nested = coroutine.create(function()
  local function inner() return coroutine.yield("in") .. "!" end
  local okp, r = pcall(function() return inner() end)
  return okp, r
end)
ok, v = coroutine.resume(nested); eq(v, "in")
local _, okp, r = coroutine.resume(nested, "back"); eq(okp, true); eq(r, "back!")

-- producer / consumer, status "normal" for the resumer
local outer
local inner = coroutine.create(function() return coroutine.status(outer) end)
outer = coroutine.create(function() local _, st = coroutine.resume(inner); return st end)
ok, v = coroutine.resume(outer); eq(v, "normal")

-- isyieldable / running on the main thread; yield outside a coroutine is an error
eq(coroutine.isyieldable(), false)
local main, ismain = coroutine.running(); eq(ismain, true)
eq(pcall(coroutine.yield, 1), false)

-- close a suspended coroutine; a never-finished coroutine is collected cleanly at exit
local c2 = coroutine.create(function() coroutine.yield(1); error("unreachable") end)
coroutine.resume(c2)
eq(coroutine.close(c2), true); eq(coroutine.status(c2), "dead")
local left = coroutine.create(function() local t = {} t.self = t coroutine.yield() end)
coroutine.resume(left)
print("ALL OK")
