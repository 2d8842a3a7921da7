// minilua — a small Lua 5.4-subset interpreter for splinterctl's `lua` verb.
//
// The reference embeds liblua5.4 and exports a `splinter` module
// (/root/reference/splinter_cli_cmd_lua.c:365-420); Lua is not installed in
// this image, so the verb runs on this self-contained tree-walking
// interpreter instead.  Supported: nil/boolean/integer/float/string/table/
// function values, closures with upvalues, varargs, multiple returns, local /
// global assignment, if/while/repeat/numeric-for/generic-for/break/return,
// method calls, string methods, integer/float arithmetic with Lua's floor
// division and modulo, bitwise ops, concatenation, and the library subset
// scripts use: print type tostring tonumber pairs ipairs next select error
// assert pcall rawget rawset rawlen unpack require load loadstring loadfile dofile,
// string.{format (incl. %q) len sub upper lower rep byte char find match gmatch gsub reverse},
// table.{insert remove concat unpack pack sort move}, math.{floor ceil abs max min sqrt exp log
// sin cos tan asin acos atan modf huge pi maxinteger mininteger random randomseed tointeger fmod
// type ult}, os.{time (incl. a date table) clock getenv date difftime remove rename tmpname
// exit}, io.{write read lines open close type stdin stdout stderr} with file methods
// (read l/L/n/a/count, write, lines, seek, flush, close), utf8.{char charpattern codepoint len
// offset codes}, goto and labels, Lua patterns (string.find / match / gmatch / gsub with
// classes, sets, quantifiers, captures, %b, %f, back-references), metatables (__index
// __newindex __call __tostring __name __len __unm __eq __lt __le, arithmetic / bitwise /
// __concat events, __pairs, __metatable) and coroutines (create resume yield status wrap
// running isyieldable close; each coroutine runs on its own thread with a strict hand-off, so
// exactly one runs at a time).  Not supported: __gc / __close / __mode, load's env argument,
// string.pack / string.dump -- documented in docs/DIVERGENCES.md.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace mlua {

struct Table;
struct Function;
struct Interp;
struct Coroutine;

struct Value {
  enum Type : uint8_t { Nil, Bool, Int, Num, Str, Tab, Fn, Co } t = Nil;
  bool b = false;
  int64_t i = 0;
  double n = 0;
  std::shared_ptr<std::string> s;
  std::shared_ptr<Table> tab;
  std::shared_ptr<Function> fn;
  std::shared_ptr<Coroutine> co;

  static Value nil() { return Value(); }
  static Value boolean(bool v) { Value x; x.t = Bool; x.b = v; return x; }
  static Value integer(int64_t v) { Value x; x.t = Int; x.i = v; return x; }
  static Value number(double v) { Value x; x.t = Num; x.n = v; return x; }
  static Value string(std::string v) { Value x; x.t = Str; x.s = std::make_shared<std::string>(std::move(v)); return x; }
  static Value table(std::shared_ptr<Table> v) { Value x; x.t = Tab; x.tab = std::move(v); return x; }
  static Value function(std::shared_ptr<Function> v) { Value x; x.t = Fn; x.fn = std::move(v); return x; }
  static Value thread(std::shared_ptr<Coroutine> v) { Value x; x.t = Co; x.co = std::move(v); return x; }
  bool truthy() const { return !(t == Nil || (t == Bool && !b)); }
  bool is_num() const { return t == Int || t == Num; }
  double as_double() const { return t == Int ? (double)i : n; }
};

struct ValueHash {
  size_t operator()(const Value& v) const;
};
struct ValueEq {
  bool operator()(const Value& a, const Value& b) const;
};

struct Heap;

// Tables and scopes register with the heap of the interpreter that is current on the thread, so
// ~Interp can break the reference cycles shared_ptr cannot collect (_G._G, a closure stored in a
// table of its own scope, ...) -- the interpreter has no tracing GC.
struct Table {
  Table();
  ~Table();
  Table(const Table&) = delete;
  Table& operator=(const Table&) = delete;
  std::vector<std::pair<Value, Value>> entries;  // insertion order (pairs / next)
  std::unordered_map<Value, size_t, ValueHash, ValueEq> index;
  std::shared_ptr<Table> meta;  // setmetatable
  Heap* heap;
  Value get(const Value& k) const;
  void set(const Value& k, const Value& v);
  int64_t length() const;
};

using Values = std::vector<Value>;
using Native = std::function<Values(Interp&, Values&)>;

struct LuaError : std::runtime_error {
  Value value;
  explicit LuaError(const std::string& m) : std::runtime_error(m), value(Value::string(m)) {}
  explicit LuaError(Value v, const std::string& m) : std::runtime_error(m), value(std::move(v)) {}
};

struct Block;
struct FuncBody;
struct Scope;

struct Function {
  Native native;
  std::shared_ptr<FuncBody> body;  // Lua closure when set
  std::shared_ptr<Scope> env;
  std::string name;
};

struct Interp {
  Interp();
  ~Interp();
  // Run a chunk of source; `args` become `...` and arg[1..n] (arg[0] = chunkname).
  Values run(const std::string& src, const std::string& chunkname, const std::vector<std::string>& args);
  void set_global(const std::string& name, Value v);
  Value global(const std::string& name) const;
  Values call(const Value& f, Values args);
  // metatable-aware table access (__index / __newindex chains), metamethod lookup, __tostring
  Value index(const Value& o, const Value& k);
  void setindex(const Value& o, const Value& k, const Value& v);
  Value metamethod(const Value& v, const char* event) const;
  std::string tostr(const Value& v);
  std::shared_ptr<Table> string_meta;  // getmetatable("") -> {__index = string}
  std::function<void(const std::string&)> out;  // print sink (default stdout)
  std::shared_ptr<Table> globals;
  std::unordered_map<std::string, Value> modules;  // require() registry
  std::shared_ptr<Scope> root;
  int depth = 0;
  int line = 0;         // line of the statement being executed (error positions)
  std::string chunk;
  Heap* heap = nullptr;       // objects created while this interpreter is current
  Heap* prev_heap = nullptr;  // restored on destruction (nested interpreters)
  // `_ENV` resolution is on once a chunk names `_ENV` or load() gets an env table: free names then
  // resolve through the innermost `_ENV` local (Lua 5.4 sec. 2.2), else the globals
  bool env_used = false;
  // tables whose metatable had __gc when it was set (Lua 5.4 sec. 2.5.3), in marking order;
  // finalized by collectgarbage() once nothing else holds them, and all of them at close
  std::vector<std::shared_ptr<Table>> finalizers;
  void run_finalizers(bool all);
  // the scope stacks of every running or suspended Lua call (roots of collectgarbage's mark phase)
  std::vector<std::vector<std::shared_ptr<Scope>>*> scope_stacks;
  std::shared_ptr<Table> registry;  // debug.getregistry()
};

std::string tostring(const Value& v);
Value make_native(const std::string& name, Native f);

}  // namespace mlua
