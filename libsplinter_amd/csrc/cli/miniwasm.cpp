// miniwasm.cpp — see miniwasm.hpp.
#include "miniwasm.hpp"

#include <cctype>
#include <cmath>
#include <cstring>
#include <limits>
#include <type_traits>

namespace mwasm {
namespace {

// ---------------------------------------------------------------------------
// opcode table (MVP + sign-extension + saturating truncation + bulk memory)
// ---------------------------------------------------------------------------
enum : uint16_t {
  OP_UNREACHABLE = 0x00, OP_NOP = 0x01, OP_BLOCK = 0x02, OP_LOOP = 0x03, OP_IF = 0x04, OP_ELSE = 0x05,
  OP_END = 0x0b, OP_BR = 0x0c, OP_BR_IF = 0x0d, OP_BR_TABLE = 0x0e, OP_RETURN = 0x0f, OP_CALL = 0x10,
  OP_CALL_INDIRECT = 0x11, OP_DROP = 0x1a, OP_SELECT = 0x1b, OP_SELECT_T = 0x1c, OP_LOCAL_GET = 0x20,
  OP_LOCAL_SET = 0x21, OP_LOCAL_TEE = 0x22, OP_GLOBAL_GET = 0x23, OP_GLOBAL_SET = 0x24, OP_MEM_SIZE = 0x3f,
  OP_MEM_GROW = 0x40, OP_I32_CONST = 0x41, OP_I64_CONST = 0x42, OP_F32_CONST = 0x43, OP_F64_CONST = 0x44,
  OP_FC = 0x100,  // 0xFC-prefixed: OP_FC + sub-opcode
};

struct OpName {
  const char* name;
  uint16_t op;
};

const OpName kOps[] = {
    {"unreachable", 0x00}, {"nop", 0x01}, {"block", 0x02}, {"loop", 0x03}, {"if", 0x04}, {"else", 0x05},
    {"end", 0x0b}, {"br", 0x0c}, {"br_if", 0x0d}, {"br_table", 0x0e}, {"return", 0x0f}, {"call", 0x10},
    {"call_indirect", 0x11}, {"drop", 0x1a}, {"select", 0x1b}, {"local.get", 0x20}, {"local.set", 0x21},
    {"local.tee", 0x22}, {"global.get", 0x23}, {"global.set", 0x24}, {"get_local", 0x20}, {"set_local", 0x21},
    {"tee_local", 0x22}, {"get_global", 0x23}, {"set_global", 0x24}, {"i32.load", 0x28}, {"i64.load", 0x29},
    {"f32.load", 0x2a}, {"f64.load", 0x2b}, {"i32.load8_s", 0x2c}, {"i32.load8_u", 0x2d}, {"i32.load16_s", 0x2e},
    {"i32.load16_u", 0x2f}, {"i64.load8_s", 0x30}, {"i64.load8_u", 0x31}, {"i64.load16_s", 0x32},
    {"i64.load16_u", 0x33}, {"i64.load32_s", 0x34}, {"i64.load32_u", 0x35}, {"i32.store", 0x36},
    {"i64.store", 0x37}, {"f32.store", 0x38}, {"f64.store", 0x39}, {"i32.store8", 0x3a}, {"i32.store16", 0x3b},
    {"i64.store8", 0x3c}, {"i64.store16", 0x3d}, {"i64.store32", 0x3e}, {"memory.size", 0x3f},
    {"memory.grow", 0x40}, {"i32.const", 0x41}, {"i64.const", 0x42}, {"f32.const", 0x43}, {"f64.const", 0x44},
    {"i32.eqz", 0x45}, {"i32.eq", 0x46}, {"i32.ne", 0x47}, {"i32.lt_s", 0x48}, {"i32.lt_u", 0x49},
    {"i32.gt_s", 0x4a}, {"i32.gt_u", 0x4b}, {"i32.le_s", 0x4c}, {"i32.le_u", 0x4d}, {"i32.ge_s", 0x4e},
    {"i32.ge_u", 0x4f}, {"i64.eqz", 0x50}, {"i64.eq", 0x51}, {"i64.ne", 0x52}, {"i64.lt_s", 0x53},
    {"i64.lt_u", 0x54}, {"i64.gt_s", 0x55}, {"i64.gt_u", 0x56}, {"i64.le_s", 0x57}, {"i64.le_u", 0x58},
    {"i64.ge_s", 0x59}, {"i64.ge_u", 0x5a}, {"f32.eq", 0x5b}, {"f32.ne", 0x5c}, {"f32.lt", 0x5d},
    {"f32.gt", 0x5e}, {"f32.le", 0x5f}, {"f32.ge", 0x60}, {"f64.eq", 0x61}, {"f64.ne", 0x62}, {"f64.lt", 0x63},
    {"f64.gt", 0x64}, {"f64.le", 0x65}, {"f64.ge", 0x66}, {"i32.clz", 0x67}, {"i32.ctz", 0x68},
    {"i32.popcnt", 0x69}, {"i32.add", 0x6a}, {"i32.sub", 0x6b}, {"i32.mul", 0x6c}, {"i32.div_s", 0x6d},
    {"i32.div_u", 0x6e}, {"i32.rem_s", 0x6f}, {"i32.rem_u", 0x70}, {"i32.and", 0x71}, {"i32.or", 0x72},
    {"i32.xor", 0x73}, {"i32.shl", 0x74}, {"i32.shr_s", 0x75}, {"i32.shr_u", 0x76}, {"i32.rotl", 0x77},
    {"i32.rotr", 0x78}, {"i64.clz", 0x79}, {"i64.ctz", 0x7a}, {"i64.popcnt", 0x7b}, {"i64.add", 0x7c},
    {"i64.sub", 0x7d}, {"i64.mul", 0x7e}, {"i64.div_s", 0x7f}, {"i64.div_u", 0x80}, {"i64.rem_s", 0x81},
    {"i64.rem_u", 0x82}, {"i64.and", 0x83}, {"i64.or", 0x84}, {"i64.xor", 0x85}, {"i64.shl", 0x86},
    {"i64.shr_s", 0x87}, {"i64.shr_u", 0x88}, {"i64.rotl", 0x89}, {"i64.rotr", 0x8a}, {"f32.abs", 0x8b},
    {"f32.neg", 0x8c}, {"f32.ceil", 0x8d}, {"f32.floor", 0x8e}, {"f32.trunc", 0x8f}, {"f32.nearest", 0x90},
    {"f32.sqrt", 0x91}, {"f32.add", 0x92}, {"f32.sub", 0x93}, {"f32.mul", 0x94}, {"f32.div", 0x95},
    {"f32.min", 0x96}, {"f32.max", 0x97}, {"f32.copysign", 0x98}, {"f64.abs", 0x99}, {"f64.neg", 0x9a},
    {"f64.ceil", 0x9b}, {"f64.floor", 0x9c}, {"f64.trunc", 0x9d}, {"f64.nearest", 0x9e}, {"f64.sqrt", 0x9f},
    {"f64.add", 0xa0}, {"f64.sub", 0xa1}, {"f64.mul", 0xa2}, {"f64.div", 0xa3}, {"f64.min", 0xa4},
    {"f64.max", 0xa5}, {"f64.copysign", 0xa6}, {"i32.wrap_i64", 0xa7}, {"i32.trunc_f32_s", 0xa8},
    {"i32.trunc_f32_u", 0xa9}, {"i32.trunc_f64_s", 0xaa}, {"i32.trunc_f64_u", 0xab}, {"i64.extend_i32_s", 0xac},
    {"i64.extend_i32_u", 0xad}, {"i64.trunc_f32_s", 0xae}, {"i64.trunc_f32_u", 0xaf}, {"i64.trunc_f64_s", 0xb0},
    {"i64.trunc_f64_u", 0xb1}, {"f32.convert_i32_s", 0xb2}, {"f32.convert_i32_u", 0xb3},
    {"f32.convert_i64_s", 0xb4}, {"f32.convert_i64_u", 0xb5}, {"f32.demote_f64", 0xb6},
    {"f64.convert_i32_s", 0xb7}, {"f64.convert_i32_u", 0xb8}, {"f64.convert_i64_s", 0xb9},
    {"f64.convert_i64_u", 0xba}, {"f64.promote_f32", 0xbb}, {"i32.reinterpret_f32", 0xbc},
    {"i64.reinterpret_f64", 0xbd}, {"f32.reinterpret_i32", 0xbe}, {"f64.reinterpret_i64", 0xbf},
    {"i32.extend8_s", 0xc0}, {"i32.extend16_s", 0xc1}, {"i64.extend8_s", 0xc2}, {"i64.extend16_s", 0xc3},
    {"i64.extend32_s", 0xc4}, {"i32.trunc_sat_f32_s", OP_FC + 0}, {"i32.trunc_sat_f32_u", OP_FC + 1},
    {"i32.trunc_sat_f64_s", OP_FC + 2}, {"i32.trunc_sat_f64_u", OP_FC + 3}, {"i64.trunc_sat_f32_s", OP_FC + 4},
    {"i64.trunc_sat_f32_u", OP_FC + 5}, {"i64.trunc_sat_f64_s", OP_FC + 6}, {"i64.trunc_sat_f64_u", OP_FC + 7},
    {"memory.copy", OP_FC + 10}, {"memory.fill", OP_FC + 11},
};

bool is_memop(uint16_t op) { return op >= 0x28 && op <= 0x3e; }

// ---------------------------------------------------------------------------
// block structure: resolve end/else targets of every block/loop/if
// ---------------------------------------------------------------------------
void resolve_blocks(std::vector<Instr>& code) {
  std::vector<uint32_t> open;
  for (uint32_t pc = 0; pc < code.size(); ++pc) {
    const uint16_t op = code[pc].op;
    if (op == OP_BLOCK || op == OP_LOOP || op == OP_IF) {
      open.push_back(pc);
    } else if (op == OP_ELSE) {
      if (open.empty() || code[open.back()].op != OP_IF) throw Error("else without if");
      code[open.back()].b = pc;
    } else if (op == OP_END) {
      if (open.empty()) continue;  // function end
      code[open.back()].a = pc;
      open.pop_back();
    }
  }
  if (!open.empty()) throw Error("unterminated block");
}

// ---------------------------------------------------------------------------
// binary decoder
// ---------------------------------------------------------------------------
struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  uint8_t u8() {
    if (p >= e) throw Error("unexpected end of module");
    return *p++;
  }
  uint64_t uleb(int bits = 64) {
    uint64_t r = 0;
    int shift = 0;
    for (;;) {
      const uint8_t b = u8();
      r |= (uint64_t)(b & 0x7f) << shift;
      shift += 7;
      if (!(b & 0x80)) break;
      if (shift > bits + 6) throw Error("bad LEB128");
    }
    return r;
  }
  int64_t sleb(int bits = 64) {
    int64_t r = 0;
    int shift = 0;
    uint8_t b;
    do {
      b = u8();
      r |= (int64_t)(b & 0x7f) << shift;
      shift += 7;
      if (shift > bits + 6) throw Error("bad LEB128");
    } while (b & 0x80);
    if (shift < 64 && (b & 0x40)) r |= -((int64_t)1 << shift);
    return r;
  }
  uint32_t u32() { return (uint32_t)uleb(32); }
  std::string name() {
    const uint32_t n = u32();
    if ((size_t)(e - p) < n) throw Error("truncated name");
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
};

void read_blocktype(Reader& r, Instr& in, const Module& m) {
  const uint8_t b = *r.p;
  if (b == 0x40) {
    r.p++;
  } else if (b == I32 || b == I64 || b == F32 || b == F64) {
    r.p++;
    in.c = 1;
  } else {
    const int64_t t = r.sleb(33);
    if (t < 0 || (size_t)t >= m.types.size()) throw Error("bad block type");
    in.c = (uint32_t)m.types[t].results.size();
    in.d = (uint32_t)m.types[t].params.size();
  }
}

std::vector<Instr> read_code(Reader& r, const Module& m, bool const_expr) {
  std::vector<Instr> code;
  int depth = 0;
  for (;;) {
    Instr in;
    uint16_t op = r.u8();
    if (op == 0xfc) op = OP_FC + (uint16_t)r.u32();
    in.op = op;
    switch (op) {
      case OP_BLOCK: case OP_LOOP: case OP_IF:
        read_blocktype(r, in, m);
        ++depth;
        break;
      case OP_END:
        code.push_back(in);
        if (depth-- == 0) return code;
        continue;
      case OP_BR: case OP_BR_IF: case OP_CALL: case OP_LOCAL_GET: case OP_LOCAL_SET: case OP_LOCAL_TEE:
      case OP_GLOBAL_GET: case OP_GLOBAL_SET:
        in.a = r.u32();
        break;
      case OP_BR_TABLE: {
        const uint32_t n = r.u32();
        for (uint32_t i = 0; i <= n; ++i) in.table.push_back(r.u32());
        break;
      }
      case OP_CALL_INDIRECT:
        in.a = r.u32();
        r.u8();  // table index 0
        break;
      case OP_SELECT_T: {
        const uint32_t n = r.u32();
        for (uint32_t i = 0; i < n; ++i) r.u8();
        in.op = OP_SELECT;
        break;
      }
      case OP_MEM_SIZE: case OP_MEM_GROW:
        r.u8();
        break;
      case OP_I32_CONST: in.b = (uint32_t)(int32_t)r.sleb(32); break;
      case OP_I64_CONST: in.b = (uint64_t)r.sleb(64); break;
      case OP_F32_CONST: {
        uint32_t v;
        if (r.e - r.p < 4) throw Error("truncated f32");
        memcpy(&v, r.p, 4);
        r.p += 4;
        in.b = v;
        break;
      }
      case OP_F64_CONST: {
        if (r.e - r.p < 8) throw Error("truncated f64");
        memcpy(&in.b, r.p, 8);
        r.p += 8;
        break;
      }
      case OP_FC + 10: r.u8(); r.u8(); break;
      case OP_FC + 11: r.u8(); break;
      default:
        if (is_memop(op)) {
          r.u32();  // align
          in.b = r.u32();
        }
        break;
    }
    if (const_expr && op != OP_I32_CONST && op != OP_I64_CONST && op != OP_F32_CONST && op != OP_F64_CONST &&
        op != OP_GLOBAL_GET)
      throw Error("non-constant initializer");
    code.push_back(std::move(in));
  }
}

}  // namespace

Module parse_binary(const std::vector<uint8_t>& bytes) {
  Module m;
  Reader r{bytes.data(), bytes.data() + bytes.size()};
  if (bytes.size() < 8 || memcmp(bytes.data(), "\0asm", 4) != 0) throw Error("not a wasm binary");
  r.p += 8;
  std::vector<uint32_t> func_types;
  while (r.p < r.e) {
    const uint8_t id = r.u8();
    const uint32_t len = r.u32();
    if ((size_t)(r.e - r.p) < len) throw Error("truncated section");
    Reader s{r.p, r.p + len};
    r.p += len;
    switch (id) {
      case 1: {  // types
        for (uint32_t n = s.u32(); n--;) {
          if (s.u8() != 0x60) throw Error("bad func type");
          FuncType t;
          for (uint32_t k = s.u32(); k--;) t.params.push_back(s.u8());
          for (uint32_t k = s.u32(); k--;) t.results.push_back(s.u8());
          m.types.push_back(t);
        }
        break;
      }
      case 2: {  // imports
        for (uint32_t n = s.u32(); n--;) {
          std::string mod = s.name(), nm = s.name();
          const uint8_t kind = s.u8();
          if (kind != 0) throw Error("only function imports are supported (" + mod + "." + nm + ")");
          m.imports.emplace_back(mod, nm);
          m.import_types.push_back(s.u32());
        }
        break;
      }
      case 3:
        for (uint32_t n = s.u32(); n--;) func_types.push_back(s.u32());
        break;
      case 4: {  // table
        for (uint32_t n = s.u32(); n--;) {
          s.u8();
          const uint8_t fl = s.u8();
          m.table_min = s.u32();
          if (fl & 1) s.u32();
        }
        break;
      }
      case 5: {  // memory
        for (uint32_t n = s.u32(); n--;) {
          const uint8_t fl = s.u8();
          m.has_memory = true;
          m.mem_min = s.u32();
          if (fl & 1) m.mem_max = s.u32();
        }
        break;
      }
      case 6: {  // globals
        for (uint32_t n = s.u32(); n--;) {
          Global g;
          g.type = s.u8();
          g.mut = s.u8() != 0;
          g.init = read_code(s, m, true);
          m.globals.push_back(g);
        }
        break;
      }
      case 7: {  // exports
        for (uint32_t n = s.u32(); n--;) {
          const std::string nm = s.name();
          Export e;
          e.kind = s.u8();
          e.index = s.u32();
          m.exports[nm] = e;
        }
        break;
      }
      case 8: m.start = s.u32(); break;
      case 9: {  // elements (MVP form: table 0, offset expr, func indices)
        for (uint32_t n = s.u32(); n--;) {
          if (s.u32() != 0) throw Error("unsupported element segment");
          Elem el;
          el.offset = read_code(s, m, true);
          for (uint32_t k = s.u32(); k--;) el.funcs.push_back(s.u32());
          m.elems.push_back(el);
        }
        break;
      }
      case 10: {  // code
        const uint32_t n = s.u32();
        if (n != func_types.size()) throw Error("function/code count mismatch");
        for (uint32_t i = 0; i < n; ++i) {
          const uint32_t sz = s.u32();
          Reader b{s.p, s.p + sz};
          s.p += sz;
          Func f;
          f.type = func_types[i];
          for (uint32_t g = b.u32(); g--;) {
            const uint32_t cnt = b.u32();
            const uint8_t t = b.u8();
            if (cnt > 65536) throw Error("too many locals");
            f.locals.insert(f.locals.end(), cnt, t);
          }
          f.code = read_code(b, m, false);
          resolve_blocks(f.code);
          m.funcs.push_back(std::move(f));
        }
        break;
      }
      case 11: {  // data (active, memory 0)
        for (uint32_t n = s.u32(); n--;) {
          const uint32_t fl = s.u32();
          if (fl == 2) s.u32();
          else if (fl != 0) throw Error("passive data segments are not supported");
          Data d;
          d.offset = read_code(s, m, true);
          const uint32_t len2 = s.u32();
          if ((size_t)(s.e - s.p) < len2) throw Error("truncated data");
          d.bytes.assign(s.p, s.p + len2);
          s.p += len2;
          m.data.push_back(d);
        }
        break;
      }
      default: break;  // custom / datacount sections
    }
  }
  if (func_types.size() != m.funcs.size()) throw Error("missing code section");
  return m;
}

// ---------------------------------------------------------------------------
// text format (WAT) parser
// ---------------------------------------------------------------------------
namespace {

struct Sx {  // s-expression node: atom (tok) or list (kids)
  bool list = false;
  bool str = false;  // quoted string atom
  std::string tok;
  std::vector<Sx> kids;
  int line = 0;
};

struct Lexer {
  const std::string& s;
  size_t i = 0;
  int line = 1;
  void skip() {
    for (;;) {
      while (i < s.size() && isspace((unsigned char)s[i])) {
        if (s[i] == '\n') ++line;
        ++i;
      }
      if (i + 1 < s.size() && s[i] == ';' && s[i + 1] == ';') {
        while (i < s.size() && s[i] != '\n') ++i;
      } else if (i + 1 < s.size() && s[i] == '(' && s[i + 1] == ';') {
        int d = 0;
        while (i + 1 < s.size()) {
          if (s[i] == '(' && s[i + 1] == ';') { ++d; i += 2; continue; }
          if (s[i] == ';' && s[i + 1] == ')') { i += 2; if (--d == 0) break; continue; }
          if (s[i] == '\n') ++line;
          ++i;
        }
      } else {
        return;
      }
    }
  }
  Sx parse() {
    skip();
    if (i >= s.size()) throw Error("unexpected end of text");
    Sx n;
    n.line = line;
    if (s[i] == '(') {
      ++i;
      n.list = true;
      for (;;) {
        skip();
        if (i >= s.size()) throw Error("unbalanced parentheses");
        if (s[i] == ')') { ++i; break; }
        n.kids.push_back(parse());
      }
    } else if (s[i] == '"') {
      ++i;
      n.str = true;
      while (i < s.size() && s[i] != '"') {
        if (s[i] == '\\' && i + 1 < s.size()) {
          const char c = s[++i];
          if (c == 'n') n.tok += '\n';
          else if (c == 't') n.tok += '\t';
          else if (c == 'r') n.tok += '\r';
          else if (c == '"' || c == '\'' || c == '\\') n.tok += c;
          else if (isxdigit((unsigned char)c) && i + 1 < s.size()) {
            n.tok += (char)std::stoi(s.substr(i, 2), nullptr, 16);
            ++i;
          } else {
            throw Error("bad string escape");
          }
          ++i;
        } else {
          n.tok += s[i++];
        }
      }
      if (i >= s.size()) throw Error("unterminated string");
      ++i;
    } else {
      const size_t b = i;
      while (i < s.size() && !isspace((unsigned char)s[i]) && s[i] != '(' && s[i] != ')' && s[i] != ';') ++i;
      n.tok = s.substr(b, i - b);
    }
    return n;
  }
};

bool head_is(const Sx& n, const char* h) { return n.list && !n.kids.empty() && !n.kids[0].list && n.kids[0].tok == h; }

uint8_t valtype(const std::string& t) {
  if (t == "i32") return I32;
  if (t == "i64") return I64;
  if (t == "f32") return F32;
  if (t == "f64") return F64;
  throw Error("unknown value type " + t);
}

std::string clean_num(const std::string& t) {
  std::string o;
  for (char c : t)
    if (c != '_') o += c;
  return o;
}

uint64_t parse_int(const std::string& t0, int bits) {
  std::string t = clean_num(t0);
  bool neg = false;
  size_t k = 0;
  if (k < t.size() && (t[k] == '-' || t[k] == '+')) neg = t[k++] == '-';
  uint64_t v;
  try {
    size_t used = 0;
    if (t.compare(k, 2, "0x") == 0) v = std::stoull(t.substr(k + 2), &used, 16), used += 2;
    else v = std::stoull(t.substr(k), &used, 10);
    if (k + used != t.size()) throw Error("bad integer " + t0);
  } catch (const std::logic_error&) {
    throw Error("bad integer " + t0);
  }
  if (neg) v = (uint64_t)(-(int64_t)v);
  if (bits == 32) v &= 0xffffffffu;
  return v;
}

double parse_float(const std::string& t0) {
  const std::string t = clean_num(t0);
  if (t == "inf" || t == "+inf") return std::numeric_limits<double>::infinity();
  if (t == "-inf") return -std::numeric_limits<double>::infinity();
  if (t.find("nan") != std::string::npos) return t[0] == '-' ? -NAN : NAN;
  try {
    return std::stod(t);  // handles decimal and C99 hex floats
  } catch (const std::logic_error&) {
    throw Error("bad float " + t0);
  }
}

struct WatCtx {
  explicit WatCtx(Module& mod) : m(mod) {}
  Module& m;
  std::map<std::string, uint32_t> funcs, globals, types;
  // per function
  std::map<std::string, uint32_t> locals;
  std::vector<std::string> labels;  // innermost last ("" if unnamed)
};

uint32_t resolve(const std::map<std::string, uint32_t>& names, const std::string& t, const char* what) {
  if (!t.empty() && t[0] == '$') {
    auto it = names.find(t);
    if (it == names.end()) throw Error(std::string("unknown ") + what + " " + t);
    return it->second;
  }
  return (uint32_t)parse_int(t, 32);
}

uint32_t label_depth(const WatCtx& c, const std::string& t) {
  if (!t.empty() && t[0] == '$') {
    for (size_t d = 0; d < c.labels.size(); ++d)
      if (c.labels[c.labels.size() - 1 - d] == t) return (uint32_t)d;
    throw Error("unknown label " + t);
  }
  return (uint32_t)parse_int(t, 32);
}

// block signature from (param ..) / (result ..) / (type ..) items starting at kids[k]
size_t block_sig(const WatCtx& c, const std::vector<Sx>& items, size_t k, Instr& in) {
  while (k < items.size() && items[k].list) {
    const Sx& it = items[k];
    if (head_is(it, "result")) in.c += (uint32_t)it.kids.size() - 1;
    else if (head_is(it, "param")) in.d += (uint32_t)it.kids.size() - 1;
    else if (head_is(it, "type")) {
      const FuncType& t = c.m.types.at(resolve(c.types, it.kids[1].tok, "type"));
      in.c = (uint32_t)t.results.size();
      in.d = (uint32_t)t.params.size();
    } else {
      break;
    }
    ++k;
  }
  return k;
}

void emit_instrs(WatCtx& c, const std::vector<Sx>& items, size_t k, std::vector<Instr>& out);

// one plain (unfolded) instruction starting at items[k]; returns next index
size_t emit_plain(WatCtx& c, const std::vector<Sx>& items, size_t k, std::vector<Instr>& out) {
  static std::map<std::string, uint16_t> names;
  if (names.empty())
    for (const auto& o : kOps) names[o.name] = o.op;
  const std::string& w = items[k].tok;
  auto it = names.find(w);
  if (it == names.end()) throw Error("unknown instruction '" + w + "' (line " + std::to_string(items[k].line) + ")");
  Instr in;
  in.op = it->second;
  ++k;
  auto atom = [&](size_t j) { return j < items.size() && !items[j].list && !items[j].str; };
  switch (in.op) {
    case OP_BLOCK: case OP_LOOP: case OP_IF: {
      std::string lab;
      if (atom(k) && items[k].tok[0] == '$') lab = items[k++].tok;
      k = block_sig(c, items, k, in);
      c.labels.push_back(lab);
      break;
    }
    case OP_END:
      if (!c.labels.empty()) c.labels.pop_back();
      if (atom(k) && items[k].tok[0] == '$') ++k;
      break;
    case OP_ELSE:
      if (atom(k) && items[k].tok[0] == '$') ++k;
      break;
    case OP_BR: case OP_BR_IF: in.a = label_depth(c, items[k++].tok); break;
    case OP_BR_TABLE:
      while (atom(k) && (items[k].tok[0] == '$' || isdigit((unsigned char)items[k].tok[0])))
        in.table.push_back(label_depth(c, items[k++].tok));
      if (in.table.empty()) throw Error("br_table needs targets");
      break;
    case OP_CALL: in.a = resolve(c.funcs, items[k++].tok, "function"); break;
    case OP_CALL_INDIRECT:
      if (k < items.size() && head_is(items[k], "type")) {
        in.a = resolve(c.types, items[k].kids[1].tok, "type");
        ++k;
      } else {
        Instr sig;
        const size_t k2 = block_sig(c, items, k, sig);
        FuncType ft;
        for (size_t j = k; j < k2; ++j)
          for (size_t q = 1; q < items[j].kids.size(); ++q)
            if (items[j].kids[q].tok[0] != '$')
              (head_is(items[j], "param") ? ft.params : ft.results).push_back(valtype(items[j].kids[q].tok));
        uint32_t ti = 0;
        for (; ti < c.m.types.size(); ++ti)
          if (c.m.types[ti] == ft) break;
        if (ti == c.m.types.size()) c.m.types.push_back(ft);
        in.a = ti;
        k = k2;
      }
      break;
    case OP_LOCAL_GET: case OP_LOCAL_SET: case OP_LOCAL_TEE: in.a = resolve(c.locals, items[k++].tok, "local"); break;
    case OP_GLOBAL_GET: case OP_GLOBAL_SET: in.a = resolve(c.globals, items[k++].tok, "global"); break;
    case OP_I32_CONST: in.b = parse_int(items[k++].tok, 32); break;
    case OP_I64_CONST: in.b = parse_int(items[k++].tok, 64); break;
    case OP_F32_CONST: {
      const float f = (float)parse_float(items[k++].tok);
      uint32_t u;
      memcpy(&u, &f, 4);
      in.b = u;
      break;
    }
    case OP_F64_CONST: {
      const double d = parse_float(items[k++].tok);
      memcpy(&in.b, &d, 8);
      break;
    }
    default:
      if (is_memop(in.op))
        while (atom(k) && (items[k].tok.rfind("offset=", 0) == 0 || items[k].tok.rfind("align=", 0) == 0)) {
          if (items[k].tok.rfind("offset=", 0) == 0) in.b = parse_int(items[k].tok.substr(7), 64);
          ++k;
        }
      break;
  }
  out.push_back(std::move(in));
  return k;
}

// folded instruction: (op imm* operands*) or (block ..) / (if .. (then ..) (else ..))
void emit_folded(WatCtx& c, const Sx& n, std::vector<Instr>& out) {
  const std::string& w = n.kids[0].tok;
  if (w == "block" || w == "loop") {
    Instr in;
    in.op = w == "block" ? OP_BLOCK : OP_LOOP;
    size_t k = 1;
    std::string lab;
    if (k < n.kids.size() && !n.kids[k].list && n.kids[k].tok[0] == '$') lab = n.kids[k++].tok;
    k = block_sig(c, n.kids, k, in);
    out.push_back(in);
    c.labels.push_back(lab);
    emit_instrs(c, n.kids, k, out);
    c.labels.pop_back();
    out.push_back(Instr(OP_END));
    return;
  }
  if (w == "if") {
    Instr in;
    in.op = OP_IF;
    size_t k = 1;
    std::string lab;
    if (k < n.kids.size() && !n.kids[k].list && n.kids[k].tok[0] == '$') lab = n.kids[k++].tok;
    k = block_sig(c, n.kids, k, in);
    // condition operands come before (then ..)
    while (k < n.kids.size() && !head_is(n.kids[k], "then")) {
      if (!n.kids[k].list) throw Error("folded if: expected (then ..)");
      emit_folded(c, n.kids[k], out);
      ++k;
    }
    out.push_back(in);
    c.labels.push_back(lab);
    if (k < n.kids.size()) emit_instrs(c, n.kids[k].kids, 1, out), ++k;
    if (k < n.kids.size() && head_is(n.kids[k], "else")) {
      out.push_back(Instr(OP_ELSE));
      emit_instrs(c, n.kids[k].kids, 1, out);
    }
    c.labels.pop_back();
    out.push_back(Instr(OP_END));
    return;
  }
  // plain op with folded operands: immediates first, then operand expressions
  size_t k = 1;
  std::vector<Sx> head{n.kids[0]};
  while (k < n.kids.size() && (!n.kids[k].list || head_is(n.kids[k], "type") || head_is(n.kids[k], "param") ||
                               head_is(n.kids[k], "result")))
    head.push_back(n.kids[k++]);
  for (; k < n.kids.size(); ++k) emit_folded(c, n.kids[k], out);
  emit_plain(c, head, 0, out);
}

void emit_instrs(WatCtx& c, const std::vector<Sx>& items, size_t k, std::vector<Instr>& out) {
  while (k < items.size()) {
    if (items[k].list) {
      emit_folded(c, items[k], out);
      ++k;
    } else {
      k = emit_plain(c, items, k, out);
    }
  }
}

std::vector<Instr> const_expr(WatCtx& c, const Sx& n) {
  std::vector<Instr> code;
  emit_folded(c, n, code);
  code.push_back(Instr(OP_END));
  return code;
}

}  // namespace

Module parse_wat(const std::string& text) {
  Lexer lx{text};
  Sx root = lx.parse();
  if (!head_is(root, "module")) throw Error("expected (module ...)");
  Module m;
  WatCtx c(m);
  size_t first = 1;
  if (first < root.kids.size() && !root.kids[first].list && root.kids[first].tok[0] == '$') ++first;
  const std::vector<Sx>& fields = root.kids;

  auto sig_of = [&](const std::vector<Sx>& items, size_t k, FuncType& ft, std::vector<std::string>* pnames,
                    size_t* next) {
    for (; k < items.size(); ++k) {
      const Sx& it = items[k];
      if (head_is(it, "type") && ft.params.empty() && ft.results.empty()) {
        ft = m.types.at(resolve(c.types, it.kids[1].tok, "type"));
        if (pnames) pnames->assign(ft.params.size(), "");
      } else if (head_is(it, "param")) {
        if (it.kids.size() >= 2 && it.kids[1].tok[0] == '$') {
          ft.params.push_back(valtype(it.kids[2].tok));
          if (pnames) pnames->push_back(it.kids[1].tok);
        } else {
          for (size_t q = 1; q < it.kids.size(); ++q) {
            ft.params.push_back(valtype(it.kids[q].tok));
            if (pnames) pnames->push_back("");
          }
        }
      } else if (head_is(it, "result")) {
        for (size_t q = 1; q < it.kids.size(); ++q) ft.results.push_back(valtype(it.kids[q].tok));
      } else {
        break;
      }
    }
    if (next) *next = k;
  };
  auto type_index = [&](const FuncType& ft) {
    for (uint32_t i = 0; i < m.types.size(); ++i)
      if (m.types[i] == ft) return i;
    m.types.push_back(ft);
    return (uint32_t)m.types.size() - 1;
  };

  // pass 1: types, imports, function / global names (indices are position based)
  uint32_t nimp = 0, nfun = 0, nglob = 0;
  for (size_t f = first; f < fields.size(); ++f) {
    const Sx& d = fields[f];
    if (head_is(d, "type")) {
      size_t k = 1;
      std::string nm;
      if (!d.kids[k].list) nm = d.kids[k++].tok;
      FuncType ft;
      sig_of(d.kids[k].kids, 1, ft, nullptr, nullptr);
      m.types.push_back(ft);
      if (!nm.empty()) c.types[nm] = (uint32_t)m.types.size() - 1;
    }
  }
  for (size_t f = first; f < fields.size(); ++f) {
    const Sx& d = fields[f];
    if (head_is(d, "import")) {
      const Sx& desc = d.kids.at(3);
      if (!head_is(desc, "func")) throw Error("only function imports are supported");
      size_t k = 1;
      if (k < desc.kids.size() && !desc.kids[k].list) c.funcs[desc.kids[k++].tok] = nimp;
      FuncType ft;
      sig_of(desc.kids, k, ft, nullptr, nullptr);
      m.imports.emplace_back(d.kids[1].tok, d.kids[2].tok);
      m.import_types.push_back(type_index(ft));
      ++nimp;
    }
  }
  for (size_t f = first; f < fields.size(); ++f) {
    const Sx& d = fields[f];
    if (head_is(d, "func")) {
      if (d.kids.size() > 1 && !d.kids[1].list) c.funcs[d.kids[1].tok] = nimp + nfun;
      ++nfun;
    } else if (head_is(d, "global")) {
      if (d.kids.size() > 1 && !d.kids[1].list) c.globals[d.kids[1].tok] = nglob;
      ++nglob;
    }
  }
  // pass 2: definitions
  for (size_t f = first; f < fields.size(); ++f) {
    const Sx& d = fields[f];
    if (head_is(d, "func")) {
      size_t k = 1;
      if (k < d.kids.size() && !d.kids[k].list) ++k;
      const uint32_t fidx = nimp + (uint32_t)m.funcs.size();
      while (k < d.kids.size() && head_is(d.kids[k], "export")) {
        m.exports[d.kids[k].kids[1].tok] = Export{0, fidx};
        ++k;
      }
      if (k < d.kids.size() && head_is(d.kids[k], "import")) throw Error("inline imports are not supported");
      FuncType ft;
      std::vector<std::string> pnames;
      sig_of(d.kids, k, ft, &pnames, &k);
      Func fn;
      fn.type = type_index(ft);
      c.locals.clear();
      c.labels.clear();
      for (uint32_t i = 0; i < pnames.size(); ++i)
        if (!pnames[i].empty()) c.locals[pnames[i]] = i;
      uint32_t li = (uint32_t)ft.params.size();
      while (k < d.kids.size() && head_is(d.kids[k], "local")) {
        const Sx& l = d.kids[k];
        if (l.kids.size() >= 3 && l.kids[1].tok[0] == '$') {
          c.locals[l.kids[1].tok] = li++;
          fn.locals.push_back(valtype(l.kids[2].tok));
        } else {
          for (size_t q = 1; q < l.kids.size(); ++q, ++li) fn.locals.push_back(valtype(l.kids[q].tok));
        }
        ++k;
      }
      emit_instrs(c, d.kids, k, fn.code);
      fn.code.push_back(Instr(OP_END));
      resolve_blocks(fn.code);
      m.funcs.push_back(std::move(fn));
    } else if (head_is(d, "memory")) {
      size_t k = 1;
      if (k < d.kids.size() && !d.kids[k].list && d.kids[k].tok[0] == '$') ++k;
      while (k < d.kids.size() && head_is(d.kids[k], "export")) m.exports[d.kids[k++].kids[1].tok] = Export{2, 0};
      m.has_memory = true;
      if (k < d.kids.size() && head_is(d.kids[k], "data")) {  // (memory (data "..."))
        Data dd;
        dd.offset = {Instr(OP_I32_CONST), Instr(OP_END)};
        for (size_t q = 1; q < d.kids[k].kids.size(); ++q) dd.bytes.insert(dd.bytes.end(), d.kids[k].kids[q].tok.begin(), d.kids[k].kids[q].tok.end());
        m.mem_min = m.mem_max = (uint32_t)((dd.bytes.size() + 65535) / 65536);
        m.data.push_back(dd);
      } else {
        if (k < d.kids.size()) m.mem_min = (uint32_t)parse_int(d.kids[k++].tok, 32);
        if (k < d.kids.size()) m.mem_max = (uint32_t)parse_int(d.kids[k++].tok, 32);
      }
    } else if (head_is(d, "data")) {
      size_t k = 1;
      if (k < d.kids.size() && !d.kids[k].list && !d.kids[k].str) ++k;  // memory index / name
      Data dd;
      if (k < d.kids.size() && head_is(d.kids[k], "memory")) ++k;
      if (k < d.kids.size() && head_is(d.kids[k], "offset")) {
        std::vector<Instr> code;
        emit_instrs(c, d.kids[k].kids, 1, code);
        code.push_back(Instr(OP_END));
        dd.offset = code;
        ++k;
      } else if (k < d.kids.size() && d.kids[k].list) {
        dd.offset = const_expr(c, d.kids[k++]);
      } else {
        throw Error("data segment needs an offset");
      }
      for (; k < d.kids.size(); ++k) dd.bytes.insert(dd.bytes.end(), d.kids[k].tok.begin(), d.kids[k].tok.end());
      m.data.push_back(dd);
    } else if (head_is(d, "global")) {
      size_t k = 1;
      if (k < d.kids.size() && !d.kids[k].list) ++k;
      while (k < d.kids.size() && head_is(d.kids[k], "export")) ++k;
      Global g;
      if (head_is(d.kids[k], "mut")) {
        g.mut = true;
        g.type = valtype(d.kids[k].kids[1].tok);
      } else {
        g.type = valtype(d.kids[k].tok);
      }
      g.init = const_expr(c, d.kids[k + 1]);
      m.globals.push_back(g);
    } else if (head_is(d, "export")) {
      const Sx& desc = d.kids.at(2);
      Export e;
      const std::string kind = desc.kids[0].tok;
      e.kind = kind == "func" ? 0 : kind == "table" ? 1 : kind == "memory" ? 2 : 3;
      e.index = e.kind == 0 ? resolve(c.funcs, desc.kids[1].tok, "function")
                : e.kind == 3 ? resolve(c.globals, desc.kids[1].tok, "global") : 0;
      m.exports[d.kids[1].tok] = e;
    } else if (head_is(d, "start")) {
      m.start = resolve(c.funcs, d.kids[1].tok, "function");
    } else if (head_is(d, "table")) {
      size_t k = 1;
      if (k < d.kids.size() && !d.kids[k].list && d.kids[k].tok[0] == '$') ++k;
      if (k < d.kids.size() && !d.kids[k].list && d.kids[k].tok != "funcref" && d.kids[k].tok != "anyfunc")
        m.table_min = (uint32_t)parse_int(d.kids[k].tok, 32);
    } else if (head_is(d, "elem")) {
      size_t k = 1;
      Elem el;
      if (k < d.kids.size() && d.kids[k].list) el.offset = const_expr(c, d.kids[k++]);
      if (k < d.kids.size() && !d.kids[k].list && d.kids[k].tok == "func") ++k;
      for (; k < d.kids.size(); ++k) el.funcs.push_back(resolve(c.funcs, d.kids[k].tok, "function"));
      m.table_min = std::max<uint32_t>(m.table_min, (uint32_t)el.funcs.size());
      m.elems.push_back(el);
    } else if (head_is(d, "type") || head_is(d, "import")) {
      // done in pass 1
    } else {
      throw Error("unsupported module field");
    }
  }
  return m;
}

Module parse_any(const std::vector<uint8_t>& bytes) {
  if (bytes.size() >= 4 && memcmp(bytes.data(), "\0asm", 4) == 0) return parse_binary(bytes);
  return parse_wat(std::string(bytes.begin(), bytes.end()));
}

// ---------------------------------------------------------------------------
// interpreter
// ---------------------------------------------------------------------------
namespace {
inline float f32(uint64_t v) {
  float f;
  const uint32_t u = (uint32_t)v;
  memcpy(&f, &u, 4);
  return f;
}
inline double f64(uint64_t v) {
  double d;
  memcpy(&d, &v, 8);
  return d;
}
inline uint64_t bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
inline uint64_t bits(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}
template <typename T>
T wasm_min(T a, T b) {
  if (std::isnan(a) || std::isnan(b)) return std::numeric_limits<T>::quiet_NaN();
  if (a == b) return std::signbit(a) ? a : b;
  return a < b ? a : b;
}
template <typename T>
T wasm_max(T a, T b) {
  if (std::isnan(a) || std::isnan(b)) return std::numeric_limits<T>::quiet_NaN();
  if (a == b) return std::signbit(a) ? b : a;
  return a > b ? a : b;
}
template <typename I, typename F>
I trunc_checked(F x) {
  if (std::isnan(x)) throw Error("invalid conversion to integer");
  const long double t = std::trunc((long double)x);
  constexpr int kBits = (int)sizeof(I) * 8;
  const long double lo = std::is_signed<I>::value ? -std::ldexp(1.0L, kBits - 1) - 1 : -1.0L;  // exclusive
  const long double hi = std::ldexp(1.0L, std::is_signed<I>::value ? kBits - 1 : kBits);      // exclusive
  if (!(t > lo && t < hi)) throw Error("integer overflow");
  return (I)t;
}
template <typename I, typename F>
I trunc_sat(F x) {
  if (std::isnan(x)) return 0;
  if (x <= (F)std::numeric_limits<I>::min()) return std::numeric_limits<I>::min();
  if (x >= (F)std::numeric_limits<I>::max()) return std::numeric_limits<I>::max();
  return (I)std::trunc(x);
}
}  // namespace

Instance::Instance(Module m, const std::map<std::string, std::pair<FuncType, HostFn>>& hosts) : m_(std::move(m)) {
  for (size_t i = 0; i < m_.imports.size(); ++i) {
    const std::string key = m_.imports[i].first + "." + m_.imports[i].second;
    auto it = hosts.find(key);
    if (it == hosts.end()) throw Error("unresolved import " + key);
    if (!(it->second.first == m_.types.at(m_.import_types[i]))) throw Error("import signature mismatch: " + key);
    host_.push_back(it->second.second);
  }
  if (m_.has_memory) {
    if (m_.mem_min > 16384) throw Error("initial memory too large");
    mem_.assign((size_t)m_.mem_min * 65536, 0);
  }
  for (const Global& g : m_.globals) globals_.push_back(eval_const(g.init));
  table_.assign(m_.table_min, -1);
  for (const Elem& e : m_.elems) {
    const uint64_t off = (uint32_t)eval_const(e.offset);
    if (off + e.funcs.size() > table_.size()) throw Error("element segment out of bounds");
    for (size_t i = 0; i < e.funcs.size(); ++i) table_[off + i] = e.funcs[i];
  }
  for (const Data& d : m_.data) {
    const uint64_t off = (uint32_t)eval_const(d.offset);
    if (off + d.bytes.size() > mem_.size()) throw Error("data segment out of bounds");
    memcpy(mem_.data() + off, d.bytes.data(), d.bytes.size());
  }
  if (m_.start >= 0) {
    std::vector<uint64_t> st;
    call((uint32_t)m_.start, st, 0);
  }
}

uint64_t Instance::eval_const(const std::vector<Instr>& code) {
  if (code.empty()) return 0;
  const Instr& in = code[0];
  if (in.op == OP_GLOBAL_GET) return globals_.at(in.a);
  return in.b;
}

uint8_t* Instance::mem_ptr(uint64_t addr, uint64_t len) {
  if (addr + len > mem_.size() || addr + len < addr) throw Error("out of bounds memory access");
  return mem_.data() + addr;
}

const FuncType& Instance::export_type(const std::string& name) const {
  auto it = m_.exports.find(name);
  if (it == m_.exports.end() || it->second.kind != 0) throw Error("no exported function '" + name + "'");
  return m_.types.at(m_.func_type(it->second.index));
}

std::vector<uint64_t> Instance::invoke(const std::string& name, const std::vector<uint64_t>& args) {
  const FuncType& t = export_type(name);
  if (args.size() != t.params.size()) throw Error("wrong number of arguments for '" + name + "'");
  std::vector<uint64_t> stack(args);
  call(m_.exports.at(name).index, stack, 0);
  return stack;
}

void Instance::call(uint32_t fidx, std::vector<uint64_t>& stack, int depth) {
  if (depth > 1000) throw Error("call stack exhausted");
  const FuncType& ft = m_.types.at(m_.func_type(fidx));
  const size_t np = ft.params.size();
  if (stack.size() < np) throw Error("stack underflow at call");
  if (fidx < m_.imports.size()) {
    std::vector<uint64_t> res(ft.results.size(), 0);
    host_[fidx](*this, stack.data() + stack.size() - np, res.data());
    stack.resize(stack.size() - np);
    stack.insert(stack.end(), res.begin(), res.end());
    return;
  }
  const Func& f = m_.funcs[fidx - m_.imports.size()];
  if (stack.size() < np) throw Error("stack underflow at call");
  std::vector<uint64_t> locals(stack.end() - np, stack.end());
  stack.resize(stack.size() - np);
  locals.resize(np + f.locals.size(), 0);
  const size_t base = stack.size();
  struct Label {
    uint32_t target;  // pc to continue at
    size_t height;    // operand stack height at entry
    uint32_t arity;   // values carried by a branch
  };
  std::vector<Label> labels;
  labels.push_back(Label{(uint32_t)f.code.size(), base, (uint32_t)ft.results.size()});
  std::vector<uint64_t>& S = stack;
  auto pop = [&]() {
    if (S.size() <= base) throw Error("stack underflow");
    const uint64_t v = S.back();
    S.pop_back();
    return v;
  };
  // operand-stack bounds are checked on every access: modules are not validated ahead of time,
  // so a malformed one must fail with an Error, never read outside the stack
  auto top = [&]() -> uint64_t {
    if (S.size() <= base) throw Error("stack underflow");
    return S.back();
  };
  auto branch = [&](uint32_t depth_, uint32_t& pc) {
    if (depth_ >= labels.size()) throw Error("bad branch depth");
    const Label L = labels[labels.size() - 1 - depth_];
    if (L.height > S.size() || S.size() - L.height < L.arity) throw Error("stack underflow at branch");
    std::vector<uint64_t> carry(S.end() - L.arity, S.end());
    S.resize(L.height);
    S.insert(S.end(), carry.begin(), carry.end());
    labels.resize(labels.size() - 1 - depth_);
    pc = L.target;
  };
  auto ea = [&](const Instr& in, uint64_t len) {
    const uint64_t addr = (uint32_t)pop() + in.b;
    return mem_ptr(addr, len);
  };
  auto ld = [&](const Instr& in, auto tag) {
    using T = decltype(tag);
    T v;
    memcpy(&v, ea(in, sizeof(T)), sizeof(T));
    return v;
  };
  auto st = [&](const Instr& in, auto v) {
    if (S.size() < base + 2) throw Error("stack underflow");
    const uint64_t addr = (uint32_t)S[S.size() - 2] + in.b;
    memcpy(mem_ptr(addr, sizeof(v)), &v, sizeof(v));
    S.resize(S.size() - 2);
  };
  uint32_t pc = 0;
  const uint32_t n = (uint32_t)f.code.size();
  while (pc < n) {
    const Instr& in = f.code[pc];
    if (step_limit && ++steps_ > step_limit) throw Error("step limit exceeded");
    uint32_t next = pc + 1;
#define BIN32(expr)                      \
  {                                      \
    const uint32_t b = (uint32_t)pop();  \
    const uint32_t a = (uint32_t)pop();  \
    S.push_back((uint32_t)(expr));       \
  }                                      \
  break;
#define BIN64(expr)              \
  {                              \
    const uint64_t b = pop();    \
    const uint64_t a = pop();    \
    S.push_back((uint64_t)(expr)); \
  }                              \
  break;
#define FBIN32(expr)                 \
  {                                  \
    const float b = f32(pop());      \
    const float a = f32(pop());      \
    S.push_back(bits((float)(expr))); \
  }                                  \
  break;
#define FBIN64(expr)                   \
  {                                    \
    const double b = f64(pop());       \
    const double a = f64(pop());       \
    S.push_back(bits((double)(expr))); \
  }                                    \
  break;
#define FCMP32(expr)            \
  {                             \
    const float b = f32(pop()); \
    const float a = f32(pop()); \
    S.push_back((expr) ? 1 : 0); \
  }                             \
  break;
#define FCMP64(expr)             \
  {                              \
    const double b = f64(pop()); \
    const double a = f64(pop()); \
    S.push_back((expr) ? 1 : 0); \
  }                              \
  break;
    switch (in.op) {
      case OP_UNREACHABLE: throw Error("unreachable executed");
      case OP_NOP: break;
      case OP_BLOCK: labels.push_back(Label{in.a + 1, S.size() - in.d, in.c}); break;
      case OP_LOOP: labels.push_back(Label{pc, S.size() - in.d, in.d}); break;
      case OP_IF: {
        const uint32_t cond = (uint32_t)pop();
        labels.push_back(Label{in.a + 1, S.size() - in.d, in.c});
        if (!cond) {
          if (in.b) next = (uint32_t)in.b + 1;  // else branch
          else { labels.pop_back(); next = in.a + 1; }
        }
        break;
      }
      case OP_ELSE: {  // end of the then-branch: skip the else body
        labels.pop_back();
        uint32_t d = 0, q = pc + 1;
        for (; q < n; ++q) {  // matching end
          const uint16_t o = f.code[q].op;
          if (o == OP_BLOCK || o == OP_LOOP || o == OP_IF) ++d;
          else if (o == OP_END) { if (d == 0) break; --d; }
        }
        next = q + 1;
        break;
      }
      case OP_END:
        if (labels.size() > 1) labels.pop_back();
        break;
      case OP_BR: branch(in.a, next); if (labels.empty()) goto done; break;
      case OP_BR_IF:
        if ((uint32_t)pop()) { branch(in.a, next); if (labels.empty()) goto done; }
        break;
      case OP_BR_TABLE: {
        const uint32_t i = (uint32_t)pop();
        branch(i < in.table.size() - 1 ? in.table[i] : in.table.back(), next);
        if (labels.empty()) goto done;
        break;
      }
      case OP_RETURN: branch((uint32_t)labels.size() - 1, next); goto done;
      case OP_CALL: call(in.a, S, depth + 1); break;
      case OP_CALL_INDIRECT: {
        const uint32_t i = (uint32_t)pop();
        if (i >= table_.size() || table_[i] < 0) throw Error("undefined table element");
        if (!(m_.types.at(m_.func_type((uint32_t)table_[i])) == m_.types.at(in.a)))
          throw Error("indirect call signature mismatch");
        call((uint32_t)table_[i], S, depth + 1);
        break;
      }
      case OP_DROP: pop(); break;
      case OP_SELECT: {
        const uint32_t c = (uint32_t)pop();
        const uint64_t b = pop(), a = pop();
        S.push_back(c ? a : b);
        break;
      }
      case OP_LOCAL_GET: S.push_back(locals.at(in.a)); break;
      case OP_LOCAL_SET: locals.at(in.a) = pop(); break;
      case OP_LOCAL_TEE: locals.at(in.a) = top(); break;
      case OP_GLOBAL_GET: S.push_back(globals_.at(in.a)); break;
      case OP_GLOBAL_SET: globals_.at(in.a) = pop(); break;
      case 0x28: S.push_back(ld(in, uint32_t())); break;
      case 0x29: S.push_back(ld(in, uint64_t())); break;
      case 0x2a: S.push_back(ld(in, uint32_t())); break;
      case 0x2b: S.push_back(ld(in, uint64_t())); break;
      case 0x2c: S.push_back((uint32_t)(int32_t)ld(in, int8_t())); break;
      case 0x2d: S.push_back((uint32_t)ld(in, uint8_t())); break;
      case 0x2e: S.push_back((uint32_t)(int32_t)ld(in, int16_t())); break;
      case 0x2f: S.push_back((uint32_t)ld(in, uint16_t())); break;
      case 0x30: S.push_back((uint64_t)(int64_t)ld(in, int8_t())); break;
      case 0x31: S.push_back((uint64_t)ld(in, uint8_t())); break;
      case 0x32: S.push_back((uint64_t)(int64_t)ld(in, int16_t())); break;
      case 0x33: S.push_back((uint64_t)ld(in, uint16_t())); break;
      case 0x34: S.push_back((uint64_t)(int64_t)ld(in, int32_t())); break;
      case 0x35: S.push_back((uint64_t)ld(in, uint32_t())); break;
      case 0x36: st(in, (uint32_t)top()); break;
      case 0x37: st(in, (uint64_t)top()); break;
      case 0x38: st(in, (uint32_t)top()); break;
      case 0x39: st(in, (uint64_t)top()); break;
      case 0x3a: st(in, (uint8_t)top()); break;
      case 0x3b: st(in, (uint16_t)top()); break;
      case 0x3c: st(in, (uint8_t)top()); break;
      case 0x3d: st(in, (uint16_t)top()); break;
      case 0x3e: st(in, (uint32_t)top()); break;
      case OP_MEM_SIZE: S.push_back(mem_.size() / 65536); break;
      case OP_MEM_GROW: {
        const uint32_t d = (uint32_t)pop();
        const uint64_t cur = mem_.size() / 65536;
        if (cur + d > m_.mem_max || cur + d > 16384) S.push_back(0xffffffffu);
        else { mem_.resize((cur + d) * 65536, 0); S.push_back((uint32_t)cur); }
        break;
      }
      case OP_I32_CONST: case OP_I64_CONST: case OP_F32_CONST: case OP_F64_CONST: S.push_back(in.b); break;
      case 0x45: S.push_back((uint32_t)pop() == 0); break;
      case 0x46: BIN32(a == b)
      case 0x47: BIN32(a != b)
      case 0x48: BIN32((int32_t)a < (int32_t)b)
      case 0x49: BIN32(a < b)
      case 0x4a: BIN32((int32_t)a > (int32_t)b)
      case 0x4b: BIN32(a > b)
      case 0x4c: BIN32((int32_t)a <= (int32_t)b)
      case 0x4d: BIN32(a <= b)
      case 0x4e: BIN32((int32_t)a >= (int32_t)b)
      case 0x4f: BIN32(a >= b)
      case 0x50: S.push_back(pop() == 0); break;
      case 0x51: BIN64(a == b)
      case 0x52: BIN64(a != b)
      case 0x53: BIN64((int64_t)a < (int64_t)b)
      case 0x54: BIN64(a < b)
      case 0x55: BIN64((int64_t)a > (int64_t)b)
      case 0x56: BIN64(a > b)
      case 0x57: BIN64((int64_t)a <= (int64_t)b)
      case 0x58: BIN64(a <= b)
      case 0x59: BIN64((int64_t)a >= (int64_t)b)
      case 0x5a: BIN64(a >= b)
      case 0x5b: FCMP32(a == b)
      case 0x5c: FCMP32(a != b)
      case 0x5d: FCMP32(a < b)
      case 0x5e: FCMP32(a > b)
      case 0x5f: FCMP32(a <= b)
      case 0x60: FCMP32(a >= b)
      case 0x61: FCMP64(a == b)
      case 0x62: FCMP64(a != b)
      case 0x63: FCMP64(a < b)
      case 0x64: FCMP64(a > b)
      case 0x65: FCMP64(a <= b)
      case 0x66: FCMP64(a >= b)
      case 0x67: { const uint32_t a = (uint32_t)pop(); S.push_back(a ? __builtin_clz(a) : 32); break; }
      case 0x68: { const uint32_t a = (uint32_t)pop(); S.push_back(a ? __builtin_ctz(a) : 32); break; }
      case 0x69: S.push_back(__builtin_popcount((uint32_t)pop())); break;
      case 0x6a: BIN32(a + b)
      case 0x6b: BIN32(a - b)
      case 0x6c: BIN32(a * b)
      case 0x6d: {
        const int32_t b = (int32_t)pop(), a = (int32_t)pop();
        if (b == 0) throw Error("integer divide by zero");
        if (a == INT32_MIN && b == -1) throw Error("integer overflow");
        S.push_back((uint32_t)(a / b));
        break;
      }
      case 0x6e: {
        const uint32_t b = (uint32_t)pop(), a = (uint32_t)pop();
        if (b == 0) throw Error("integer divide by zero");
        S.push_back(a / b);
        break;
      }
      case 0x6f: {
        const int32_t b = (int32_t)pop(), a = (int32_t)pop();
        if (b == 0) throw Error("integer divide by zero");
        S.push_back((uint32_t)(b == -1 ? 0 : a % b));
        break;
      }
      case 0x70: {
        const uint32_t b = (uint32_t)pop(), a = (uint32_t)pop();
        if (b == 0) throw Error("integer divide by zero");
        S.push_back(a % b);
        break;
      }
      case 0x71: BIN32(a & b)
      case 0x72: BIN32(a | b)
      case 0x73: BIN32(a ^ b)
      case 0x74: BIN32(a << (b & 31))
      case 0x75: BIN32((int32_t)a >> (b & 31))
      case 0x76: BIN32(a >> (b & 31))
      case 0x77: BIN32((a << (b & 31)) | (a >> ((32 - (b & 31)) & 31)))
      case 0x78: BIN32((a >> (b & 31)) | (a << ((32 - (b & 31)) & 31)))
      case 0x79: { const uint64_t a = pop(); S.push_back(a ? __builtin_clzll(a) : 64); break; }
      case 0x7a: { const uint64_t a = pop(); S.push_back(a ? __builtin_ctzll(a) : 64); break; }
      case 0x7b: S.push_back(__builtin_popcountll(pop())); break;
      case 0x7c: BIN64(a + b)
      case 0x7d: BIN64(a - b)
      case 0x7e: BIN64(a * b)
      case 0x7f: {
        const int64_t b = (int64_t)pop(), a = (int64_t)pop();
        if (b == 0) throw Error("integer divide by zero");
        if (a == INT64_MIN && b == -1) throw Error("integer overflow");
        S.push_back((uint64_t)(a / b));
        break;
      }
      case 0x80: {
        const uint64_t b = pop(), a = pop();
        if (b == 0) throw Error("integer divide by zero");
        S.push_back(a / b);
        break;
      }
      case 0x81: {
        const int64_t b = (int64_t)pop(), a = (int64_t)pop();
        if (b == 0) throw Error("integer divide by zero");
        S.push_back((uint64_t)(b == -1 ? 0 : a % b));
        break;
      }
      case 0x82: {
        const uint64_t b = pop(), a = pop();
        if (b == 0) throw Error("integer divide by zero");
        S.push_back(a % b);
        break;
      }
      case 0x83: BIN64(a & b)
      case 0x84: BIN64(a | b)
      case 0x85: BIN64(a ^ b)
      case 0x86: BIN64(a << (b & 63))
      case 0x87: BIN64((int64_t)a >> (b & 63))
      case 0x88: BIN64(a >> (b & 63))
      case 0x89: BIN64((a << (b & 63)) | (a >> ((64 - (b & 63)) & 63)))
      case 0x8a: BIN64((a >> (b & 63)) | (a << ((64 - (b & 63)) & 63)))
      case 0x8b: S.push_back(bits(std::fabs(f32(pop())))); break;
      case 0x8c: S.push_back(pop() ^ 0x80000000u); break;
      case 0x8d: S.push_back(bits(std::ceil(f32(pop())))); break;
      case 0x8e: S.push_back(bits(std::floor(f32(pop())))); break;
      case 0x8f: S.push_back(bits(std::trunc(f32(pop())))); break;
      case 0x90: S.push_back(bits(std::nearbyint(f32(pop())))); break;
      case 0x91: S.push_back(bits(std::sqrt(f32(pop())))); break;
      case 0x92: FBIN32(a + b)
      case 0x93: FBIN32(a - b)
      case 0x94: FBIN32(a * b)
      case 0x95: FBIN32(a / b)
      case 0x96: FBIN32(wasm_min(a, b))
      case 0x97: FBIN32(wasm_max(a, b))
      case 0x98: FBIN32(std::copysign(a, b))
      case 0x99: S.push_back(bits(std::fabs(f64(pop())))); break;
      case 0x9a: S.push_back(pop() ^ 0x8000000000000000ull); break;
      case 0x9b: S.push_back(bits(std::ceil(f64(pop())))); break;
      case 0x9c: S.push_back(bits(std::floor(f64(pop())))); break;
      case 0x9d: S.push_back(bits(std::trunc(f64(pop())))); break;
      case 0x9e: S.push_back(bits(std::nearbyint(f64(pop())))); break;
      case 0x9f: S.push_back(bits(std::sqrt(f64(pop())))); break;
      case 0xa0: FBIN64(a + b)
      case 0xa1: FBIN64(a - b)
      case 0xa2: FBIN64(a * b)
      case 0xa3: FBIN64(a / b)
      case 0xa4: FBIN64(wasm_min(a, b))
      case 0xa5: FBIN64(wasm_max(a, b))
      case 0xa6: FBIN64(std::copysign(a, b))
      case 0xa7: S.push_back((uint32_t)pop()); break;
      case 0xa8: S.push_back((uint32_t)trunc_checked<int32_t>(f32(pop()))); break;
      case 0xa9: S.push_back(trunc_checked<uint32_t>(f32(pop()))); break;
      case 0xaa: S.push_back((uint32_t)trunc_checked<int32_t>(f64(pop()))); break;
      case 0xab: S.push_back(trunc_checked<uint32_t>(f64(pop()))); break;
      case 0xac: S.push_back((uint64_t)(int64_t)(int32_t)(uint32_t)pop()); break;
      case 0xad: S.push_back((uint64_t)(uint32_t)pop()); break;
      case 0xae: S.push_back((uint64_t)trunc_checked<int64_t>(f32(pop()))); break;
      case 0xaf: S.push_back(trunc_checked<uint64_t>(f32(pop()))); break;
      case 0xb0: S.push_back((uint64_t)trunc_checked<int64_t>(f64(pop()))); break;
      case 0xb1: S.push_back(trunc_checked<uint64_t>(f64(pop()))); break;
      case 0xb2: S.push_back(bits((float)(int32_t)(uint32_t)pop())); break;
      case 0xb3: S.push_back(bits((float)(uint32_t)pop())); break;
      case 0xb4: S.push_back(bits((float)(int64_t)pop())); break;
      case 0xb5: S.push_back(bits((float)pop())); break;
      case 0xb6: S.push_back(bits((float)f64(pop()))); break;
      case 0xb7: S.push_back(bits((double)(int32_t)(uint32_t)pop())); break;
      case 0xb8: S.push_back(bits((double)(uint32_t)pop())); break;
      case 0xb9: S.push_back(bits((double)(int64_t)pop())); break;
      case 0xba: S.push_back(bits((double)pop())); break;
      case 0xbb: S.push_back(bits((double)f32(pop()))); break;
      case 0xbc: case 0xbe: S.push_back((uint32_t)pop()); break;
      case 0xbd: case 0xbf: break;  // same bits
      case 0xc0: S.push_back((uint32_t)(int32_t)(int8_t)pop()); break;
      case 0xc1: S.push_back((uint32_t)(int32_t)(int16_t)pop()); break;
      case 0xc2: S.push_back((uint64_t)(int64_t)(int8_t)pop()); break;
      case 0xc3: S.push_back((uint64_t)(int64_t)(int16_t)pop()); break;
      case 0xc4: S.push_back((uint64_t)(int64_t)(int32_t)pop()); break;
      case OP_FC + 0: S.push_back((uint32_t)trunc_sat<int32_t>(f32(pop()))); break;
      case OP_FC + 1: S.push_back(trunc_sat<uint32_t>(f32(pop()))); break;
      case OP_FC + 2: S.push_back((uint32_t)trunc_sat<int32_t>(f64(pop()))); break;
      case OP_FC + 3: S.push_back(trunc_sat<uint32_t>(f64(pop()))); break;
      case OP_FC + 4: S.push_back((uint64_t)trunc_sat<int64_t>(f32(pop()))); break;
      case OP_FC + 5: S.push_back(trunc_sat<uint64_t>(f32(pop()))); break;
      case OP_FC + 6: S.push_back((uint64_t)trunc_sat<int64_t>(f64(pop()))); break;
      case OP_FC + 7: S.push_back(trunc_sat<uint64_t>(f64(pop()))); break;
      case OP_FC + 10: {
        const uint32_t len = (uint32_t)pop(), src = (uint32_t)pop(), dst = (uint32_t)pop();
        memmove(mem_ptr(dst, len), mem_ptr(src, len), len);
        break;
      }
      case OP_FC + 11: {
        const uint32_t len = (uint32_t)pop(), val = (uint32_t)pop(), dst = (uint32_t)pop();
        memset(mem_ptr(dst, len), (int)(val & 0xff), len);
        break;
      }
      default: throw Error("unsupported opcode " + std::to_string(in.op));
    }
#undef BIN32
#undef BIN64
#undef FBIN32
#undef FBIN64
#undef FCMP32
#undef FCMP64
    pc = next;
  }
done:
  // function results are the top `results` values above the frame base
  if (S.size() < base + ft.results.size()) throw Error("missing function results");
  if (S.size() < ft.results.size()) throw Error("stack underflow at return");
  std::vector<uint64_t> res(S.end() - ft.results.size(), S.end());
  S.resize(base);
  S.insert(S.end(), res.begin(), res.end());
}

}  // namespace mwasm
