// miniwasm — a small WebAssembly (MVP) interpreter for the CLI `wasm` verb.
//
// The reference runs modules on WasmEdge with a `splinter` host module
// (/root/reference/splinter_cli_cmd_wasm.c:20-77: `get`, `set`; :85-143 VM
// dispatch).  WasmEdge is not available in this image, so the verb carries
// its own interpreter: binary modules (.wasm, MVP: i32/i64/f32/f64, memory,
// globals, tables + call_indirect, imports of host functions) and the text
// format (WAT, the subset the reference's own test.wasm uses and the usual
// folded / flat instruction forms), decoded into one IR and run by a
// stack interpreter with branch targets resolved at load time.
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace mwasm {

enum VT : uint8_t { I32 = 0x7f, I64 = 0x7e, F32 = 0x7d, F64 = 0x7c };

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct FuncType {
  std::vector<uint8_t> params, results;
  bool operator==(const FuncType& o) const { return params == o.params && results == o.results; }
};

// One decoded instruction.  a/b: immediates (index, branch target, memarg
// offset, constant bits); for block/loop/if: a = pc of the matching end,
// b = pc of else (if), c = block arity (results), d = params.
struct Instr {
  Instr() = default;
  explicit Instr(uint16_t o) : op(o) {}
  uint16_t op = 0;
  uint32_t a = 0, c = 0, d = 0;
  uint64_t b = 0;
  std::vector<uint32_t> table;  // br_table targets (last = default)
};

struct Func {
  uint32_t type = 0;
  std::vector<uint8_t> locals;  // declared locals (after params)
  std::vector<Instr> code;
};

struct Global {
  uint8_t type = I32;
  bool mut = false;
  std::vector<Instr> init;
};

struct Data {
  std::vector<Instr> offset;
  std::vector<uint8_t> bytes;
};

struct Elem {
  std::vector<Instr> offset;
  std::vector<uint32_t> funcs;
};

struct Export {
  uint8_t kind = 0;  // 0 func, 1 table, 2 memory, 3 global
  uint32_t index = 0;
};

struct Module {
  std::vector<FuncType> types;
  std::vector<std::pair<std::string, std::string>> imports;  // imported functions (module, name)
  std::vector<uint32_t> import_types;
  std::vector<Func> funcs;                                    // defined functions
  bool has_memory = false;
  uint32_t mem_min = 0, mem_max = 65536;
  uint32_t table_min = 0;
  std::vector<Global> globals;
  std::vector<Data> data;
  std::vector<Elem> elems;
  std::map<std::string, Export> exports;
  int64_t start = -1;
  uint32_t func_type(uint32_t idx) const {
    return idx < imports.size() ? import_types[idx] : funcs.at(idx - imports.size()).type;
  }
};

Module parse_binary(const std::vector<uint8_t>& bytes);
Module parse_wat(const std::string& text);
// binary if it starts with "\0asm", else text
Module parse_any(const std::vector<uint8_t>& bytes);

class Instance;
// host function: args in, results out (values as raw bits); throw Error to trap
using HostFn = std::function<void(Instance&, const uint64_t* args, uint64_t* results)>;

class Instance {
 public:
  // hosts: "module.name" -> (type, fn); every import must resolve
  Instance(Module m, const std::map<std::string, std::pair<FuncType, HostFn>>& hosts);
  std::vector<uint64_t> invoke(const std::string& export_name, const std::vector<uint64_t>& args = {});
  const FuncType& export_type(const std::string& export_name) const;
  std::vector<uint8_t>& memory() { return mem_; }
  // bounds-checked guest memory access for host functions
  uint8_t* mem_ptr(uint64_t addr, uint64_t len);
  uint64_t steps() const { return steps_; }
  uint64_t step_limit = 0;  // 0 = unlimited

 private:
  void call(uint32_t fidx, std::vector<uint64_t>& stack, int depth);
  uint64_t eval_const(const std::vector<Instr>& code);
  Module m_;
  std::vector<uint8_t> mem_;
  std::vector<uint64_t> globals_;
  std::vector<int64_t> table_;
  std::vector<HostFn> host_;
  uint64_t steps_ = 0;
};

}  // namespace mwasm
