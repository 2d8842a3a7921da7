// minilua.cpp — lexer, parser, tree-walking evaluator and standard library
// subset for the `lua` verb (see minilua.hpp for scope).
#include "minilua.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <random>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <unistd.h>
#include <cerrno>

namespace mlua {

// ------------------------------------------------------------ values ------
static bool float_is_int(double d, int64_t* out) {
  if (std::isfinite(d) && d == std::floor(d) && d >= -9.2233720368547758e18 && d < 9.2233720368547758e18) {
    *out = (int64_t)d;
    return true;
  }
  return false;
}

size_t ValueHash::operator()(const Value& v) const {
  switch (v.t) {
    case Value::Nil: return 0;
    case Value::Bool: return v.b ? 1 : 2;
    case Value::Int: return std::hash<int64_t>()(v.i);
    case Value::Num: {
      int64_t i;
      if (float_is_int(v.n, &i)) return std::hash<int64_t>()(i);
      return std::hash<double>()(v.n);
    }
    case Value::Str: return std::hash<std::string>()(*v.s);
    case Value::Tab: return std::hash<const void*>()(v.tab.get());
    case Value::Fn: return std::hash<const void*>()(v.fn.get());
    case Value::Co: return std::hash<const void*>()(v.co.get());
  }
  return 0;
}

static bool raw_equal(const Value& a, const Value& b) {
  if (a.is_num() && b.is_num()) {
    if (a.t == Value::Int && b.t == Value::Int) return a.i == b.i;
    return a.as_double() == b.as_double();
  }
  if (a.t != b.t) return false;
  switch (a.t) {
    case Value::Nil: return true;
    case Value::Bool: return a.b == b.b;
    case Value::Str: return *a.s == *b.s;
    case Value::Tab: return a.tab == b.tab;
    case Value::Fn: return a.fn == b.fn;
    case Value::Co: return a.co == b.co;
    default: return false;
  }
}

bool ValueEq::operator()(const Value& a, const Value& b) const { return raw_equal(a, b); }

static Value norm_key(const Value& k) {
  int64_t i;
  if (k.t == Value::Num && float_is_int(k.n, &i)) return Value::integer(i);
  return k;
}

Value Table::get(const Value& k) const {
  auto it = index.find(norm_key(k));
  return it == index.end() ? Value() : entries[it->second].second;
}

void Table::set(const Value& k0, const Value& v) {
  if (k0.t == Value::Nil) throw LuaError("table index is nil");
  if (k0.t == Value::Num && std::isnan(k0.n)) throw LuaError("table index is NaN");
  const Value k = norm_key(k0);
  auto it = index.find(k);
  if (it != index.end()) {
    entries[it->second].second = v;
  } else if (v.t != Value::Nil) {
    index.emplace(k, entries.size());
    entries.emplace_back(k, v);
  }
}

int64_t Table::length() const {
  int64_t n = 0;
  while (get(Value::integer(n + 1)).t != Value::Nil) ++n;
  return n;
}

static std::string fmt_number(double d) {  // lua_Number format "%.14g", ".0" when it reads as an integer
  if (std::isinf(d)) return d > 0 ? "inf" : "-inf";
  if (std::isnan(d)) return "nan";
  char b[64];
  snprintf(b, sizeof b, "%.14g", d);
  if (strspn(b, "-0123456789") == strlen(b)) strcat(b, ".0");
  return b;
}

std::string tostring(const Value& v) {
  char b[64];
  switch (v.t) {
    case Value::Nil: return "nil";
    case Value::Bool: return v.b ? "true" : "false";
    case Value::Int: snprintf(b, sizeof b, "%lld", (long long)v.i); return b;
    case Value::Num: return fmt_number(v.n);
    case Value::Str: return *v.s;
    case Value::Tab: snprintf(b, sizeof b, "table: %p", (void*)v.tab.get()); return b;
    case Value::Fn: snprintf(b, sizeof b, "function: %p", (void*)v.fn.get()); return b;
    case Value::Co: snprintf(b, sizeof b, "thread: %p", (void*)v.co.get()); return b;
  }
  return "?";
}

static const char* type_name(const Value& v) {
  switch (v.t) {
    case Value::Nil: return "nil";
    case Value::Bool: return "boolean";
    case Value::Int:
    case Value::Num: return "number";
    case Value::Str: return "string";
    case Value::Tab: return "table";
    case Value::Fn: return "function";
    case Value::Co: return "thread";
  }
  return "?";
}

Value make_native(const std::string& name, Native f) {
  auto fn = std::make_shared<Function>();
  fn->native = std::move(f);
  fn->name = name;
  return Value::function(fn);
}

// string -> number (Lua coercion rules, decimal/hex ints and floats)
static bool str2num(const std::string& s0, Value* out) {
  std::string s = s0;
  size_t a = s.find_first_not_of(" \t\n\r\f\v"), b = s.find_last_not_of(" \t\n\r\f\v");
  if (a == std::string::npos) return false;
  s = s.substr(a, b - a + 1);
  const char* c = s.c_str();
  char* end = nullptr;
  bool neg = false;
  const char* p = c;
  if (*p == '-' || *p == '+') { neg = *p == '-'; ++p; }
  if (p[0] == '0' && (p[1] == 'x' || p[1] == 'X')) {
    errno = 0;
    unsigned long long u = strtoull(p + 2, &end, 16);
    if (*end == 0 && end != p + 2) { *out = Value::integer(neg ? -(int64_t)u : (int64_t)u); return true; }
    return false;
  }
  bool isint = s.find_first_of(".eEnN") == std::string::npos;
  if (isint) {
    errno = 0;
    long long v = strtoll(c, &end, 10);
    if (*end == 0 && errno == 0) { *out = Value::integer(v); return true; }
  }
  double d = strtod(c, &end);
  if (*end == 0 && end != c) { *out = Value::number(d); return true; }
  return false;
}

static bool tonum(const Value& v, Value* out) {
  if (v.is_num()) { *out = v; return true; }
  if (v.t == Value::Str) return str2num(*v.s, out);
  return false;
}

static int64_t toint_strict(const Value& v, const char* what) {
  Value n;
  if (!tonum(v, &n)) throw LuaError(std::string("bad argument (number expected, got ") + type_name(v) + ") to " + what);
  if (n.t == Value::Int) return n.i;
  int64_t i;
  if (float_is_int(n.n, &i)) return i;
  throw LuaError(std::string("number has no integer representation in ") + what);
}

// ------------------------------------------------------------ lexer -------
enum Tok {
  T_EOF, T_NAME, T_NUMBER, T_STRING,
  T_AND, T_BREAK, T_DO, T_ELSE, T_ELSEIF, T_END, T_FALSE, T_FOR, T_FUNCTION, T_IF, T_IN, T_LOCAL, T_NIL, T_NOT,
  T_OR, T_REPEAT, T_RETURN, T_THEN, T_TRUE, T_UNTIL, T_WHILE, T_GOTO,
  T_EQ, T_NE, T_LE, T_GE, T_CONCAT, T_DOTS, T_IDIV, T_SHL, T_SHR, T_DBCOLON,
  T_CHAR  // single-char token in `ch`
};

struct Token {
  Tok t = T_EOF;
  std::string s;
  Value num;
  char ch = 0;
  int line = 1;
};

struct Lexer {
  const std::string& src;
  size_t p = 0;
  int line = 1;
  std::string chunk;
  explicit Lexer(const std::string& s, std::string c) : src(s), chunk(std::move(c)) {}

  [[noreturn]] void err(const std::string& m) { throw LuaError(chunk + ":" + std::to_string(line) + ": " + m); }
  char at(size_t k = 0) const { return p + k < src.size() ? src[p + k] : 0; }

  bool long_bracket(std::string* out) {  // at '[': [[...]] or [==[...]==]
    size_t q = p + 1;
    int level = 0;
    while (q < src.size() && src[q] == '=') { ++level; ++q; }
    if (q >= src.size() || src[q] != '[') return false;
    q++;
    if (q < src.size() && src[q] == '\n') { ++line; ++q; }
    std::string close = "]" + std::string((size_t)level, '=') + "]";
    size_t e = src.find(close, q);
    if (e == std::string::npos) err("unfinished long string");
    for (size_t k = q; k < e; ++k) if (src[k] == '\n') ++line;
    if (out) *out = src.substr(q, e - q);
    p = e + close.size();
    return true;
  }

  void skip() {
    for (;;) {
      char c = at();
      if (c == '\n') { ++line; ++p; }
      else if (c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v') ++p;
      else if (c == '-' && at(1) == '-') {
        p += 2;
        if (at() == '[' && long_bracket(nullptr)) continue;
        while (at() && at() != '\n') ++p;
      } else if (c == '#' && p == 0 && at(1) == '!') {
        while (at() && at() != '\n') ++p;
      } else break;
    }
  }

  Token next() {
    skip();
    Token t;
    t.line = line;
    char c = at();
    if (!c) { t.t = T_EOF; return t; }
    if (isalpha((unsigned char)c) || c == '_') {
      size_t s = p;
      while (isalnum((unsigned char)at()) || at() == '_') ++p;
      t.s = src.substr(s, p - s);
      static const std::unordered_map<std::string, Tok> kw = {
          {"and", T_AND}, {"break", T_BREAK}, {"do", T_DO}, {"else", T_ELSE}, {"elseif", T_ELSEIF}, {"end", T_END},
          {"false", T_FALSE}, {"for", T_FOR}, {"function", T_FUNCTION}, {"if", T_IF}, {"in", T_IN},
          {"local", T_LOCAL}, {"nil", T_NIL}, {"not", T_NOT}, {"or", T_OR}, {"repeat", T_REPEAT},
          {"return", T_RETURN}, {"then", T_THEN}, {"true", T_TRUE}, {"until", T_UNTIL}, {"while", T_WHILE}, {"goto", T_GOTO}};
      auto it = kw.find(t.s);
      t.t = it == kw.end() ? T_NAME : it->second;
      return t;
    }
    if (isdigit((unsigned char)c) || (c == '.' && isdigit((unsigned char)at(1)))) {
      size_t s = p;
      if (c == '0' && (at(1) == 'x' || at(1) == 'X')) {
        p += 2;
        while (isxdigit((unsigned char)at()) || at() == '.') ++p;
      } else {
        while (isdigit((unsigned char)at()) || at() == '.') ++p;
        if (at() == 'e' || at() == 'E') {
          ++p;
          if (at() == '+' || at() == '-') ++p;
          while (isdigit((unsigned char)at())) ++p;
        }
      }
      t.t = T_NUMBER;
      if (!str2num(src.substr(s, p - s), &t.num)) err("malformed number near '" + src.substr(s, p - s) + "'");
      return t;
    }
    if (c == '"' || c == '\'') {
      const char q = c;
      ++p;
      std::string out;
      while (at() != q) {
        char d = at();
        if (!d || d == '\n') err("unfinished string");
        if (d == '\\') {
          ++p;
          char e = at();
          ++p;
          switch (e) {
            case 'n': out += '\n'; break;
            case 't': out += '\t'; break;
            case 'r': out += '\r'; break;
            case 'a': out += '\a'; break;
            case 'b': out += '\b'; break;
            case 'f': out += '\f'; break;
            case 'v': out += '\v'; break;
            case '\\': out += '\\'; break;
            case '"': out += '"'; break;
            case '\'': out += '\''; break;
            case '\n': out += '\n'; ++line; break;
            case 'x': {
              int v = (int)strtol(src.substr(p, 2).c_str(), nullptr, 16);
              p += 2;
              out += (char)v;
              break;
            }
            case 'z': while (isspace((unsigned char)at())) { if (at() == '\n') ++line; ++p; } break;
            default:
              if (isdigit((unsigned char)e)) {
                int v = e - '0';
                for (int k = 0; k < 2 && isdigit((unsigned char)at()); ++k) v = v * 10 + (at() - '0'), ++p;
                out += (char)v;
              } else {
                err(std::string("invalid escape sequence '\\") + e + "'");
              }
          }
        } else {
          out += d;
          ++p;
        }
      }
      ++p;
      t.t = T_STRING;
      t.s = out;
      return t;
    }
    if (c == '[' && (at(1) == '[' || at(1) == '=')) {
      std::string s;
      if (long_bracket(&s)) { t.t = T_STRING; t.s = s; return t; }
    }
    auto two = [&](char a, char b, Tok k) {
      if (c == a && at(1) == b) { p += 2; t.t = k; return true; }
      return false;
    };
    if (c == '.' && at(1) == '.' && at(2) == '.') { p += 3; t.t = T_DOTS; return t; }
    if (two('=', '=', T_EQ) || two('~', '=', T_NE) || two('<', '=', T_LE) || two('>', '=', T_GE) ||
        two('.', '.', T_CONCAT) || two('/', '/', T_IDIV) || two('<', '<', T_SHL) || two('>', '>', T_SHR) ||
        two(':', ':', T_DBCOLON))
      return t;
    t.t = T_CHAR;
    t.ch = c;
    ++p;
    return t;
  }
};

// ------------------------------------------------------------ AST ---------
struct Expr;
struct Stat;
using ExprP = std::shared_ptr<Expr>;
using StatP = std::shared_ptr<Stat>;

struct Block {
  std::vector<StatP> stats;
};

struct FuncBody {
  std::vector<std::string> params;
  bool vararg = false;
  std::shared_ptr<Block> block;
  std::string name;
};

enum ExprKind { E_NIL, E_TRUE, E_FALSE, E_NUM, E_STR, E_VARARG, E_FUNC, E_TABLE, E_BIN, E_UN, E_NAME, E_INDEX,
                E_CALL, E_METHOD, E_PAREN, E_AND, E_OR };

struct Expr {
  ExprKind k;
  Value lit;
  std::string name;
  int op = 0;  // token / char code
  ExprP a, b;
  std::vector<ExprP> args;
  std::shared_ptr<FuncBody> fn;
  // table constructor: items (key may be null = positional)
  std::vector<std::pair<ExprP, ExprP>> items;
  int line = 0;
};

enum StatKind { S_LOCAL, S_ASSIGN, S_CALL, S_DO, S_WHILE, S_REPEAT, S_IF, S_NUMFOR, S_GENFOR, S_RETURN, S_BREAK,
                S_LOCALFUNC, S_GOTO, S_LABEL };

struct Stat {
  StatKind k;
  std::vector<std::string> names;
  std::vector<ExprP> targets, exprs;
  ExprP e;
  std::shared_ptr<Block> body;
  std::vector<ExprP> conds;
  std::vector<std::shared_ptr<Block>> blocks;
  std::shared_ptr<Block> els;
  std::shared_ptr<FuncBody> fn;
  std::vector<int> attribs;  // S_LOCAL: per name 0, 1 <const>, 2 <close>
  int line = 0;
};

// ------------------------------------------------------------ parser ------
struct Parser {
  Lexer lx;
  Token cur, ahead;
  bool has_ahead = false;
  Parser(const std::string& src, const std::string& chunk) : lx(src, chunk) { cur = lx.next(); }

  [[noreturn]] void err(const std::string& m) {
    throw LuaError(lx.chunk + ":" + std::to_string(cur.line) + ": " + m + " near '" + show(cur) + "'");
  }
  static std::string show(const Token& t) {
    switch (t.t) {
      case T_EOF: return "<eof>";
      case T_NAME: case T_STRING: return t.s;
      case T_NUMBER: return tostring(t.num);
      case T_CHAR: return std::string(1, t.ch);
      default: return "token";
    }
  }
  void advance() {
    if (has_ahead) { cur = ahead; has_ahead = false; }
    else cur = lx.next();
  }
  const Token& peek() {
    if (!has_ahead) { ahead = lx.next(); has_ahead = true; }
    return ahead;
  }
  bool is(char c) const { return cur.t == T_CHAR && cur.ch == c; }
  bool accept(char c) { if (is(c)) { advance(); return true; } return false; }
  bool accept(Tok t) { if (cur.t == t) { advance(); return true; } return false; }
  void expect(char c) { if (!accept(c)) err(std::string("'") + c + "' expected"); }
  void expect(Tok t, const char* what) { if (!accept(t)) err(std::string("'") + what + "' expected"); }
  std::string name() {
    if (cur.t != T_NAME) err("<name> expected");
    std::string s = cur.s;
    advance();
    return s;
  }

  bool block_end() const {
    return cur.t == T_EOF || cur.t == T_END || cur.t == T_ELSE || cur.t == T_ELSEIF || cur.t == T_UNTIL;
  }

  std::shared_ptr<Block> block() {
    auto b = std::make_shared<Block>();
    while (!block_end()) {
      if (cur.t == T_RETURN) {
        auto s = std::make_shared<Stat>();
        s->k = S_RETURN;
        s->line = cur.line;
        advance();
        if (!block_end() && !is(';')) s->exprs = exprlist();
        accept(';');
        b->stats.push_back(s);
        if (!block_end()) err("'end' expected after return");
        break;
      }
      if (accept(';')) continue;
      b->stats.push_back(statement());
    }
    return b;
  }

  std::shared_ptr<FuncBody> funcbody(const std::string& nm, bool method) {
    auto f = std::make_shared<FuncBody>();
    f->name = nm;
    if (method) f->params.push_back("self");
    expect('(');
    if (!is(')')) {
      do {
        if (accept(T_DOTS)) { f->vararg = true; break; }
        f->params.push_back(name());
      } while (accept(','));
    }
    expect(')');
    f->block = block();
    expect(T_END, "end");
    return f;
  }

  StatP statement() {
    auto s = std::make_shared<Stat>();
    s->line = cur.line;
    switch (cur.t) {
      case T_IF: {
        advance();
        s->k = S_IF;
        s->conds.push_back(expr());
        expect(T_THEN, "then");
        s->blocks.push_back(block());
        while (cur.t == T_ELSEIF) {
          advance();
          s->conds.push_back(expr());
          expect(T_THEN, "then");
          s->blocks.push_back(block());
        }
        if (accept(T_ELSE)) s->els = block();
        expect(T_END, "end");
        return s;
      }
      case T_WHILE:
        advance();
        s->k = S_WHILE;
        s->e = expr();
        expect(T_DO, "do");
        s->body = block();
        expect(T_END, "end");
        return s;
      case T_DO:
        advance();
        s->k = S_DO;
        s->body = block();
        expect(T_END, "end");
        return s;
      case T_REPEAT:
        advance();
        s->k = S_REPEAT;
        s->body = block();
        expect(T_UNTIL, "until");
        s->e = expr();
        return s;
      case T_FOR: {
        advance();
        std::string n1 = name();
        if (accept('=')) {
          s->k = S_NUMFOR;
          s->names.push_back(n1);
          s->exprs.push_back(expr());
          expect(',');
          s->exprs.push_back(expr());
          if (accept(',')) s->exprs.push_back(expr());
        } else {
          s->k = S_GENFOR;
          s->names.push_back(n1);
          while (accept(',')) s->names.push_back(name());
          expect(T_IN, "in");
          s->exprs = exprlist();
        }
        expect(T_DO, "do");
        s->body = block();
        expect(T_END, "end");
        return s;
      }
      case T_FUNCTION: {
        advance();
        // funcname: Name {'.' Name} [':' Name]
        auto target = std::make_shared<Expr>();
        target->k = E_NAME;
        target->name = name();
        std::string full = target->name;
        bool method = false;
        while (is('.') || is(':')) {
          method = is(':');
          advance();
          auto idx = std::make_shared<Expr>();
          idx->k = E_INDEX;
          idx->a = target;
          idx->b = std::make_shared<Expr>();
          idx->b->k = E_STR;
          idx->b->lit = Value::string(name());
          full += (method ? ":" : ".") + *idx->b->lit.s;
          target = idx;
          if (method) break;
        }
        s->k = S_ASSIGN;
        s->targets.push_back(target);
        auto fe = std::make_shared<Expr>();
        fe->k = E_FUNC;
        fe->fn = funcbody(full, method);
        s->exprs.push_back(fe);
        return s;
      }
      case T_LOCAL:
        advance();
        if (accept(T_FUNCTION)) {
          s->k = S_LOCALFUNC;
          s->names.push_back(name());
          s->fn = funcbody(s->names[0], false);
          return s;
        }
        s->k = S_LOCAL;
        do {
          s->names.push_back(name());
          int at = 0;
          if (accept('<')) {
            const std::string a = name();
            if (a == "const") at = 1;
            else if (a == "close") at = 2;
            else err("unknown attribute '" + a + "'");
            expect('>');
          }
          s->attribs.push_back(at);
        } while (accept(','));
        {
          int closes = 0;
          for (int a : s->attribs) closes += a == 2;
          if (closes > 1) err("multiple to-be-closed variables in local list");
        }
        if (accept('=')) s->exprs = exprlist();
        return s;
      case T_BREAK:
        advance();
        s->k = S_BREAK;
        return s;
      case T_GOTO:
        advance();
        s->k = S_GOTO;
        s->names.push_back(name());
        return s;
      case T_DBCOLON:
        advance();
        s->k = S_LABEL;
        s->names.push_back(name());
        if (!accept(T_DBCOLON)) err("'::' expected");
        return s;
      default: break;
    }
    // exprstat: call or assignment
    ExprP e = suffixedexp();
    if (is('=') || is(',')) {
      s->k = S_ASSIGN;
      s->targets.push_back(e);
      while (accept(',')) s->targets.push_back(suffixedexp());
      expect('=');
      s->exprs = exprlist();
      for (auto& t : s->targets)
        if (t->k != E_NAME && t->k != E_INDEX) err("syntax error (cannot assign)");
      return s;
    }
    if (e->k != E_CALL && e->k != E_METHOD) err("syntax error");
    s->k = S_CALL;
    s->e = e;
    return s;
  }

  std::vector<ExprP> exprlist() {
    std::vector<ExprP> v;
    v.push_back(expr());
    while (accept(',')) v.push_back(expr());
    return v;
  }

  ExprP primaryexp() {
    auto e = std::make_shared<Expr>();
    e->line = cur.line;
    if (cur.t == T_NAME) {
      e->k = E_NAME;
      e->name = cur.s;
      advance();
      return e;
    }
    if (accept('(')) {
      e->k = E_PAREN;
      e->a = expr();
      expect(')');
      return e;
    }
    err("unexpected symbol");
  }

  std::vector<ExprP> callargs() {
    std::vector<ExprP> args;
    if (cur.t == T_STRING) {
      auto s = std::make_shared<Expr>();
      s->k = E_STR;
      s->lit = Value::string(cur.s);
      advance();
      args.push_back(s);
    } else if (is('{')) {
      args.push_back(tablecons());
    } else {
      expect('(');
      if (!is(')')) args = exprlist();
      expect(')');
    }
    return args;
  }

  ExprP suffixedexp() {
    ExprP e = primaryexp();
    for (;;) {
      const int line = cur.line;
      if (accept('.')) {
        auto x = std::make_shared<Expr>();
        x->k = E_INDEX;
        x->a = e;
        x->b = std::make_shared<Expr>();
        x->b->k = E_STR;
        x->b->lit = Value::string(name());
        x->line = line;
        e = x;
      } else if (accept('[')) {
        auto x = std::make_shared<Expr>();
        x->k = E_INDEX;
        x->a = e;
        x->b = expr();
        x->line = line;
        expect(']');
        e = x;
      } else if (accept(':')) {
        auto x = std::make_shared<Expr>();
        x->k = E_METHOD;
        x->a = e;
        x->name = name();
        x->args = callargs();
        x->line = line;
        e = x;
      } else if (is('(') || is('{') || cur.t == T_STRING) {
        auto x = std::make_shared<Expr>();
        x->k = E_CALL;
        x->a = e;
        x->args = callargs();
        x->line = line;
        e = x;
      } else {
        return e;
      }
    }
  }

  ExprP tablecons() {
    auto t = std::make_shared<Expr>();
    t->k = E_TABLE;
    t->line = cur.line;
    expect('{');
    while (!is('}')) {
      if (accept('[')) {
        ExprP k = expr();
        expect(']');
        expect('=');
        t->items.emplace_back(k, expr());
      } else if (cur.t == T_NAME && peek().t == T_CHAR && peek().ch == '=') {
        auto k = std::make_shared<Expr>();
        k->k = E_STR;
        k->lit = Value::string(cur.s);
        advance();
        advance();
        t->items.emplace_back(k, expr());
      } else {
        t->items.emplace_back(nullptr, expr());
      }
      if (!accept(',') && !accept(';')) break;
    }
    expect('}');
    return t;
  }

  ExprP simpleexp() {
    auto e = std::make_shared<Expr>();
    e->line = cur.line;
    switch (cur.t) {
      case T_NUMBER: e->k = E_NUM; e->lit = cur.num; advance(); return e;
      case T_STRING: e->k = E_STR; e->lit = Value::string(cur.s); advance(); return e;
      case T_NIL: e->k = E_NIL; advance(); return e;
      case T_TRUE: e->k = E_TRUE; advance(); return e;
      case T_FALSE: e->k = E_FALSE; advance(); return e;
      case T_DOTS: e->k = E_VARARG; advance(); return e;
      case T_FUNCTION: advance(); e->k = E_FUNC; e->fn = funcbody("anonymous", false); return e;
      default: break;
    }
    if (is('{')) return tablecons();
    return suffixedexp();
  }

  // binary precedence (left, right) as in lparser.c
  static bool binop(const Token& t, int* op, int* l, int* r) {
    struct P { int op, l, r; };
    P p{0, 0, 0};
    if (t.t == T_CHAR) {
      switch (t.ch) {
        case '+': p = {'+', 10, 10}; break;
        case '-': p = {'-', 10, 10}; break;
        case '*': p = {'*', 11, 11}; break;
        case '/': p = {'/', 11, 11}; break;
        case '%': p = {'%', 11, 11}; break;
        case '^': p = {'^', 14, 13}; break;
        case '&': p = {'&', 6, 6}; break;
        case '|': p = {'|', 4, 4}; break;
        case '~': p = {'~', 5, 5}; break;
        case '<': p = {'<', 3, 3}; break;
        case '>': p = {'>', 3, 3}; break;
        default: return false;
      }
    } else {
      switch (t.t) {
        case T_IDIV: p = {T_IDIV + 256, 11, 11}; break;
        case T_CONCAT: p = {T_CONCAT + 256, 9, 8}; break;
        case T_SHL: p = {T_SHL + 256, 7, 7}; break;
        case T_SHR: p = {T_SHR + 256, 7, 7}; break;
        case T_EQ: p = {T_EQ + 256, 3, 3}; break;
        case T_NE: p = {T_NE + 256, 3, 3}; break;
        case T_LE: p = {T_LE + 256, 3, 3}; break;
        case T_GE: p = {T_GE + 256, 3, 3}; break;
        case T_AND: p = {T_AND + 256, 2, 2}; break;
        case T_OR: p = {T_OR + 256, 1, 1}; break;
        default: return false;
      }
    }
    *op = p.op;
    *l = p.l;
    *r = p.r;
    return true;
  }

  ExprP expr(int limit = 0) {
    ExprP left;
    const int line = cur.line;
    if (cur.t == T_NOT || is('-') || is('#') || is('~')) {
      int op = cur.t == T_NOT ? T_NOT + 256 : cur.ch;
      advance();
      auto u = std::make_shared<Expr>();
      u->k = E_UN;
      u->op = op;
      u->a = expr(12);
      u->line = line;
      left = u;
    } else {
      left = simpleexp();
    }
    int op, l, r;
    while (binop(cur, &op, &l, &r) && l > limit) {
      advance();
      ExprP right = expr(r);
      auto b = std::make_shared<Expr>();
      b->line = line;
      if (op == T_AND + 256) b->k = E_AND;
      else if (op == T_OR + 256) b->k = E_OR;
      else b->k = E_BIN;
      b->op = op;
      b->a = left;
      b->b = right;
      left = b;
    }
    return left;
  }
};

// ------------------------------------------------------------ evaluator ---
struct Scope {
  Scope();
  ~Scope();
  std::unordered_map<std::string, std::shared_ptr<Value>> vars;
  std::shared_ptr<Scope> parent;
  Values varargs;
  bool has_varargs = false;
  Heap* heap;
  std::vector<Value> tbc;  // to-be-closed values of this block (`local x <close>`), in declaration order
};

struct Heap {
  std::unordered_set<Table*> tables;
  std::unordered_set<Scope*> scopes;
};
static thread_local Heap* t_heap = nullptr;

Table::Table() : heap(t_heap) { if (heap) heap->tables.insert(this); }
Table::~Table() { if (heap) heap->tables.erase(this); }
Scope::Scope() : heap(t_heap) { if (heap) heap->scopes.insert(this); }
Scope::~Scope() { if (heap) heap->scopes.erase(this); }

// F_GOTO: a `goto` looking for its label; every enclosing block searches its own statements
// (Lua 5.4: a label is visible in the block that defines it and in nested blocks, functions excluded)
enum Flow { F_NORMAL, F_BREAK, F_RETURN, F_GOTO };

struct Exec {
  Interp& I;
  Values ret;
  std::string go_label;  // the label a pending F_GOTO looks for

  // run b's statements from index `from`; a goto whose label is in b continues at the label
  Flow run_stats(const std::shared_ptr<Block>& b, const std::shared_ptr<Scope>& sc) {
    Flow f = F_NORMAL;
    for (size_t i = 0; i < b->stats.size(); ++i) {
      f = exec(b->stats[i], sc);
      if (f == F_GOTO) {
        size_t j = 0;
        for (; j < b->stats.size(); ++j)
          if (b->stats[j]->k == S_LABEL && b->stats[j]->names[0] == go_label) break;
        if (j < b->stats.size()) {
          i = j;  // the loop's ++i runs the statement after the label
          f = F_NORMAL;
          continue;
        }
      }
      if (f != F_NORMAL) break;
    }
    return f;
  }
  explicit Exec(Interp& in) : I(in) { I.scope_stacks.push_back(&live); }
  ~Exec() {
    auto& v = I.scope_stacks;
    for (size_t i = v.size(); i-- > 0;)
      if (v[i] == &live) {
        v.erase(v.begin() + (long)i);
        break;
      }
  }
  Exec(const Exec&) = delete;
  Exec& operator=(const Exec&) = delete;

  std::shared_ptr<Value> lookup(Scope* s, const std::string& n) {
    for (; s; s = s->parent.get()) {
      auto it = s->vars.find(n);
      if (it != s->vars.end()) return it->second;
    }
    return nullptr;
  }

  [[noreturn]] void rt(const Expr* e, const std::string& m) {
    throw LuaError(I.chunk + ":" + std::to_string(e && e->line ? e->line : I.line) + ": " + m);
  }

  Value index(const Value& o, const Value& k, const Expr* e) {
    if (o.t != Value::Tab && o.t != Value::Str)
      rt(e, std::string("attempt to index a ") + type_name(o) + " value" +
                (e && e->a && e->a->k == E_NAME ? " (variable '" + e->a->name + "')" : ""));
    return I.index(o, k);
  }

  // binary metamethod (__add, __concat, __lt, ...): the left operand's, else the right one's
  bool meta_bin(const char* ev, const Value& a, const Value& b, Value* out) {
    Value h = I.metamethod(a, ev);
    if (h.t == Value::Nil) h = I.metamethod(b, ev);
    if (h.t == Value::Nil) return false;
    Values r = I.call(h, {a, b});
    *out = r.empty() ? Value() : r[0];
    return true;
  }

  Values eval_multi(const ExprP& e, Scope* s) {
    if (e->k == E_CALL || e->k == E_METHOD) return call_expr(e.get(), s);
    if (e->k == E_VARARG) {
      for (Scope* x = s; x; x = x->parent.get())
        if (x->has_varargs) return x->varargs;
      return {};
    }
    return {eval(e, s)};
  }

  Values eval_list(const std::vector<ExprP>& es, Scope* s) {
    Values out;
    for (size_t i = 0; i < es.size(); ++i) {
      if (i + 1 == es.size()) {
        Values m = eval_multi(es[i], s);
        out.insert(out.end(), m.begin(), m.end());
      } else {
        out.push_back(eval(es[i], s));
      }
    }
    return out;
  }

  Values call_expr(const Expr* e, Scope* s) {
    Value f;
    Values args;
    if (e->k == E_METHOD) {
      Value obj = eval(e->a, s);
      f = index(obj, Value::string(e->name), e);
      if (f.t != Value::Fn && I.metamethod(f, "__call").t == Value::Nil)
        rt(e, "attempt to call a " + std::string(type_name(f)) + " value (method '" + e->name + "')");
      args.push_back(obj);
    } else {
      f = eval(e->a, s);
      if (f.t != Value::Fn && I.metamethod(f, "__call").t == Value::Nil) {
        std::string what = e->a->k == E_NAME ? " (global '" + e->a->name + "')" : "";
        rt(e, std::string("attempt to call a ") + type_name(f) + " value" + what);
      }
    }
    Values rest = eval_list(e->args, s);
    args.insert(args.end(), rest.begin(), rest.end());
    return I.call(f, std::move(args));
  }

  static Value arith(int op, const Value& a0, const Value& b0, const Expr* e, Exec& ex) {
    Value a, b;
    if (!tonum(a0, &a) || !tonum(b0, &b))
      ex.rt(e, std::string("attempt to perform arithmetic on a ") + type_name(tonum(a0, &a) ? b0 : a0) + " value");
    const bool ints = a.t == Value::Int && b.t == Value::Int;
    switch (op) {
      case '+': return ints ? Value::integer((int64_t)((uint64_t)a.i + (uint64_t)b.i)) : Value::number(a.as_double() + b.as_double());
      case '-': return ints ? Value::integer((int64_t)((uint64_t)a.i - (uint64_t)b.i)) : Value::number(a.as_double() - b.as_double());
      case '*': return ints ? Value::integer((int64_t)((uint64_t)a.i * (uint64_t)b.i)) : Value::number(a.as_double() * b.as_double());
      case '/': return Value::number(a.as_double() / b.as_double());
      case '^': return Value::number(std::pow(a.as_double(), b.as_double()));
      case '%':
        if (ints) {
          if (b.i == 0) ex.rt(e, "attempt to perform 'n%%0'");
          int64_t m = a.i % b.i;
          if (m != 0 && ((m ^ b.i) < 0)) m += b.i;
          return Value::integer(m);
        } else {
          double x = a.as_double(), y = b.as_double(), m = std::fmod(x, y);
          if (m != 0 && ((m < 0) != (y < 0))) m += y;
          return Value::number(m);
        }
      default:  // floor division
        if (ints) {
          if (b.i == 0) ex.rt(e, "attempt to perform 'n//0'");
          int64_t q = a.i / b.i;
          if ((a.i % b.i != 0) && ((a.i < 0) != (b.i < 0))) --q;
          return Value::integer(q);
        }
        return Value::number(std::floor(a.as_double() / b.as_double()));
    }
  }

  static bool less(const Value& a, const Value& b, const Expr* e, Exec& ex, bool orequal) {
    if (a.is_num() && b.is_num()) {
      if (a.t == Value::Int && b.t == Value::Int) return orequal ? a.i <= b.i : a.i < b.i;
      return orequal ? a.as_double() <= b.as_double() : a.as_double() < b.as_double();
    }
    if (a.t == Value::Str && b.t == Value::Str) return orequal ? *a.s <= *b.s : *a.s < *b.s;
    ex.rt(e, std::string("attempt to compare ") + type_name(a) + " with " + type_name(b));
  }

  Value eval(const ExprP& e, Scope* s) {
    switch (e->k) {
      case E_NIL: return Value();
      case E_TRUE: return Value::boolean(true);
      case E_FALSE: return Value::boolean(false);
      case E_NUM:
      case E_STR: return e->lit;
      case E_VARARG: {
        Values v = eval_multi(e, s);
        return v.empty() ? Value() : v[0];
      }
      case E_FUNC: {
        auto f = std::make_shared<Function>();
        f->body = e->fn;
        f->name = e->fn->name;
        // capture the defining scope (shared): closures see later updates of upvalues
        f->env = scope_ptr(s);
        return Value::function(f);
      }
      case E_TABLE: {
        auto t = std::make_shared<Table>();
        int64_t n = 1;
        for (size_t i = 0; i < e->items.size(); ++i) {
          auto& it = e->items[i];
          if (it.first) {
            t->set(eval(it.first, s), eval(it.second, s));
          } else if (i + 1 == e->items.size()) {
            for (auto& v : eval_multi(it.second, s)) t->set(Value::integer(n++), v);
          } else {
            t->set(Value::integer(n++), eval(it.second, s));
          }
        }
        return Value::table(t);
      }
      case E_AND: {
        Value a = eval(e->a, s);
        return a.truthy() ? eval(e->b, s) : a;
      }
      case E_OR: {
        Value a = eval(e->a, s);
        return a.truthy() ? a : eval(e->b, s);
      }
      case E_UN: {
        Value a = eval(e->a, s);
        Value mr;
        switch (e->op) {
          case T_NOT + 256: return Value::boolean(!a.truthy());
          case '-': {
            Value n;
            if (!tonum(a, &n)) {
              if (meta_bin("__unm", a, a, &mr)) return mr;
              rt(e.get(), std::string("attempt to perform arithmetic on a ") + type_name(a) + " value");
            }
            return n.t == Value::Int ? Value::integer((int64_t)(0 - (uint64_t)n.i)) : Value::number(-n.n);
          }
          case '#':
            if (a.t == Value::Str) return Value::integer((int64_t)a.s->size());
            if (meta_bin("__len", a, a, &mr)) return mr;
            if (a.t == Value::Tab) return Value::integer(a.tab->length());
            rt(e.get(), std::string("attempt to get length of a ") + type_name(a) + " value");
          case '~':
            if (a.t == Value::Tab && meta_bin("__bnot", a, a, &mr)) return mr;
            return Value::integer(~toint_strict(a, "bitwise not"));
        }
        rt(e.get(), "bad unary operator");
      }
      case E_BIN: {
        Value a = eval(e->a, s), b = eval(e->b, s);
        const int op = e->op;
        if (a.t == Value::Tab || b.t == Value::Tab) {  // metamethods (tables only carry metatables)
          const char* ev = nullptr;
          bool swap = false, negate = false;
          switch (op) {
            case '+': ev = "__add"; break;
            case '-': ev = "__sub"; break;
            case '*': ev = "__mul"; break;
            case '/': ev = "__div"; break;
            case '%': ev = "__mod"; break;
            case '^': ev = "__pow"; break;
            case T_IDIV + 256: ev = "__idiv"; break;
            case '&': ev = "__band"; break;
            case '|': ev = "__bor"; break;
            case '~': ev = "__bxor"; break;
            case T_SHL + 256: ev = "__shl"; break;
            case T_SHR + 256: ev = "__shr"; break;
            case T_CONCAT + 256: ev = "__concat"; break;
            case '<': ev = "__lt"; break;
            case T_LE + 256: ev = "__le"; break;
            case '>': ev = "__lt"; swap = true; break;
            case T_GE + 256: ev = "__le"; swap = true; break;
            case T_EQ + 256:
            case T_NE + 256:
              if (a.t == Value::Tab && b.t == Value::Tab && !raw_equal(a, b)) ev = "__eq";
              negate = op == T_NE + 256;
              break;
          }
          Value mr;
          if (ev && meta_bin(ev, swap ? b : a, swap ? a : b, &mr)) {
            const bool cmp = op == '<' || op == '>' || op == T_LE + 256 || op == T_GE + 256 || op == T_EQ + 256 ||
                             op == T_NE + 256;
            if (!cmp) return mr;
            return Value::boolean(negate ? !mr.truthy() : mr.truthy());
          }
        }
        switch (op) {
          case '+': case '-': case '*': case '/': case '%': case '^': case T_IDIV + 256:
            return arith(op == T_IDIV + 256 ? 'i' : op, a, b, e.get(), *this);
          case T_CONCAT + 256: {
            auto str = [&](const Value& v) -> std::string {
              if (v.t == Value::Str) return *v.s;
              if (v.is_num()) return tostring(v);
              rt(e.get(), std::string("attempt to concatenate a ") + type_name(v) + " value");
            };
            return Value::string(str(a) + str(b));
          }
          case T_EQ + 256: return Value::boolean(raw_equal(a, b));
          case T_NE + 256: return Value::boolean(!raw_equal(a, b));
          case '<': return Value::boolean(less(a, b, e.get(), *this, false));
          case T_LE + 256: return Value::boolean(less(a, b, e.get(), *this, true));
          case '>': return Value::boolean(less(b, a, e.get(), *this, false));
          case T_GE + 256: return Value::boolean(less(b, a, e.get(), *this, true));
          case '&': return Value::integer(toint_strict(a, "bitwise and") & toint_strict(b, "bitwise and"));
          case '|': return Value::integer(toint_strict(a, "bitwise or") | toint_strict(b, "bitwise or"));
          case '~': return Value::integer(toint_strict(a, "bitwise xor") ^ toint_strict(b, "bitwise xor"));
          case T_SHL + 256: {
            int64_t x = toint_strict(a, "shift"), n = toint_strict(b, "shift");
            if (n <= -64 || n >= 64) return Value::integer(0);
            return Value::integer(n >= 0 ? (int64_t)((uint64_t)x << n) : (int64_t)((uint64_t)x >> -n));
          }
          case T_SHR + 256: {
            int64_t x = toint_strict(a, "shift"), n = toint_strict(b, "shift");
            if (n <= -64 || n >= 64) return Value::integer(0);
            return Value::integer(n >= 0 ? (int64_t)((uint64_t)x >> n) : (int64_t)((uint64_t)x << -n));
          }
        }
        rt(e.get(), "bad binary operator");
      }
      case E_NAME: {
        if (auto c = lookup(s, e->name)) return *c;
        if (I.env_used) {
          if (auto env = lookup(s, "_ENV")) {
            if (env->t != Value::Tab && env->t != Value::Str)
              rt(e.get(), std::string("attempt to index a ") + type_name(*env) + " value (upvalue '_ENV')");
            return I.index(*env, Value::string(e->name));
          }
          if (e->name == "_ENV") return Value::table(I.globals);
        }
        return I.globals->get(Value::string(e->name));
      }
      case E_INDEX: return index(eval(e->a, s), eval(e->b, s), e.get());
      case E_CALL:
      case E_METHOD: {
        Values v = call_expr(e.get(), s);
        return v.empty() ? Value() : v[0];
      }
      case E_PAREN: return eval(e->a, s);
    }
    return Value();
  }

  // scopes are held by shared_ptr so closures can keep them alive
  std::vector<std::shared_ptr<Scope>> live;
  std::shared_ptr<Scope> scope_ptr(Scope* s) {
    for (auto it = live.rbegin(); it != live.rend(); ++it)
      if (it->get() == s) return *it;
    return nullptr;
  }
  std::shared_ptr<Scope> push(const std::shared_ptr<Scope>& parent) {
    auto sc = std::make_shared<Scope>();
    sc->parent = parent;
    live.push_back(sc);
    return sc;
  }
  void pop() { live.pop_back(); }

  void assign(const ExprP& t, const Value& v, Scope* s) {
    if (t->k == E_NAME) {
      if (auto c = lookup(s, t->name)) {
        *c = v;
      } else if (I.env_used && t->name != "_ENV") {
        if (auto env = lookup(s, "_ENV")) {
          if (env->t != Value::Tab) rt(t.get(), std::string("attempt to index a ") + type_name(*env) + " value (upvalue '_ENV')");
          I.setindex(*env, Value::string(t->name), v);
        } else {
          I.globals->set(Value::string(t->name), v);
        }
      } else {
        I.globals->set(Value::string(t->name), v);
      }
    } else {
      Value o = eval(t->a, s);
      if (o.t != Value::Tab && I.metamethod(o, "__newindex").t == Value::Nil)
        rt(t.get(), std::string("attempt to index a ") + type_name(o) + " value");
      I.setindex(o, eval(t->b, s), v);
    }
  }

  // `local x <close>`: the block's to-be-closed values get __close(value, error) in reverse order
  // when the block ends -- normally, by break / return / goto, or by an error (Lua 5.4 sec. 3.3.8).
  // An error in a closing method replaces the block's error and the remaining methods still run.
  void close_tbc(Scope* sc, Value err, bool errored) {
    std::unique_ptr<LuaError> raised;
    while (!sc->tbc.empty()) {
      Value v = std::move(sc->tbc.back());
      sc->tbc.pop_back();
      Value h = I.metamethod(v, "__close");
      if (h.t == Value::Nil) continue;
      try {
        I.call(h, {v, errored ? err : Value()});
      } catch (LuaError& e) {
        err = e.value;
        errored = true;
        raised = std::make_unique<LuaError>(e.value, e.what());
      }
    }
    if (raised) throw LuaError(raised->value, raised->what());
  }
  Flow run_closing(const std::shared_ptr<Block>& b, const std::shared_ptr<Scope>& sc) {
    Flow f = F_NORMAL;
    try {
      f = run_stats(b, sc);
    } catch (LuaError& e) {
      if (sc->tbc.empty()) throw;
      close_tbc(sc.get(), e.value, true);
      throw;
    } catch (...) {  // a coroutine being closed: its pending variables are closed too
      if (!sc->tbc.empty()) close_tbc(sc.get(), Value(), false);
      throw;
    }
    if (!sc->tbc.empty()) close_tbc(sc.get(), Value(), false);
    return f;
  }
  Flow exec_block(const std::shared_ptr<Block>& b, const std::shared_ptr<Scope>& parent) {
    auto sc = push(parent);
    Flow f = F_NORMAL;
    try {
      f = run_closing(b, sc);
    } catch (...) {
      pop();
      throw;
    }
    pop();
    return f;
  }

  Flow exec(const StatP& st, const std::shared_ptr<Scope>& sc) {
    Scope* s = sc.get();
    I.line = st->line;
    switch (st->k) {
      case S_LOCAL: {
        Values v = eval_list(st->exprs, s);
        for (size_t i = 0; i < st->names.size(); ++i) {
          Value x = i < v.size() ? v[i] : Value();
          if (st->attribs.size() > i && st->attribs[i] == 2 && x.truthy()) {  // nil / false: nothing to close
            if (I.metamethod(x, "__close").t == Value::Nil)
              rt(nullptr, "variable '" + st->names[i] + "' got a non-closable value");
            s->tbc.push_back(x);
          }
          s->vars[st->names[i]] = std::make_shared<Value>(std::move(x));
        }
        return F_NORMAL;
      }
      case S_LOCALFUNC: {
        auto cell = std::make_shared<Value>();
        s->vars[st->names[0]] = cell;
        auto f = std::make_shared<Function>();
        f->body = st->fn;
        f->name = st->names[0];
        f->env = sc;
        *cell = Value::function(f);
        return F_NORMAL;
      }
      case S_ASSIGN: {
        Values v = eval_list(st->exprs, s);
        for (size_t i = 0; i < st->targets.size(); ++i) assign(st->targets[i], i < v.size() ? v[i] : Value(), s);
        return F_NORMAL;
      }
      case S_CALL: call_expr(st->e.get(), s); return F_NORMAL;
      case S_DO: return exec_block(st->body, sc);
      case S_WHILE:
        while (eval(st->e, s).truthy()) {
          Flow f = exec_block(st->body, sc);
          if (f == F_BREAK) break;
          if (f == F_RETURN || f == F_GOTO) return f;
        }
        return F_NORMAL;
      case S_REPEAT:
        for (;;) {
          // the until-condition sees the body's locals
          auto inner = push(sc);
          Flow f = F_NORMAL;
          bool done = false;
          try {
            f = run_closing(st->body, inner);
            if (f == F_NORMAL) done = eval(st->e, inner.get()).truthy();
          } catch (...) {
            pop();
            throw;
          }
          pop();
          if (f == F_BREAK) break;
          if (f == F_RETURN || f == F_GOTO) return f;
          if (done) break;
        }
        return F_NORMAL;
      case S_IF:
        for (size_t i = 0; i < st->conds.size(); ++i)
          if (eval(st->conds[i], s).truthy()) return exec_block(st->blocks[i], sc);
        if (st->els) return exec_block(st->els, sc);
        return F_NORMAL;
      case S_NUMFOR: {
        Value a = eval(st->exprs[0], s), b = eval(st->exprs[1], s);
        Value c = st->exprs.size() > 2 ? eval(st->exprs[2], s) : Value::integer(1);
        Value x, y, z;
        if (!tonum(a, &x) || !tonum(b, &y) || !tonum(c, &z)) rt(st->exprs[0].get(), "'for' values must be numbers");
        if (x.t == Value::Int && y.t == Value::Int && z.t == Value::Int) {
          if (z.i == 0) rt(st->exprs[0].get(), "'for' step is zero");
          for (int64_t i = x.i; z.i > 0 ? i <= y.i : i >= y.i; i += z.i) {
            auto body = push(sc);
            body->vars[st->names[0]] = std::make_shared<Value>(Value::integer(i));
            pop();
            Flow f = exec_block(st->body, body);
            if (f == F_BREAK) break;
            if (f == F_RETURN || f == F_GOTO) return f;
            if ((z.i > 0 && i > INT64_MAX - z.i) || (z.i < 0 && i < INT64_MIN - z.i)) break;
          }
        } else {
          double i0 = x.as_double(), lim = y.as_double(), stp = z.as_double();
          if (stp == 0) rt(st->exprs[0].get(), "'for' step is zero");
          for (double i = i0; stp > 0 ? i <= lim : i >= lim; i += stp) {
            auto body = push(sc);
            body->vars[st->names[0]] = std::make_shared<Value>(Value::number(i));
            pop();
            Flow f = exec_block(st->body, body);
            if (f == F_BREAK) break;
            if (f == F_RETURN || f == F_GOTO) return f;
          }
        }
        return F_NORMAL;
      }
      case S_GENFOR: {
        Values it = eval_list(st->exprs, s);
        Value f = it.size() > 0 ? it[0] : Value(), state = it.size() > 1 ? it[1] : Value(),
              ctl = it.size() > 2 ? it[2] : Value();
        if (f.t != Value::Fn) rt(st->exprs[0].get(), std::string("attempt to call a ") + type_name(f) + " value");
        for (;;) {
          Values r = I.call(f, {state, ctl});
          if (r.empty() || r[0].t == Value::Nil) break;
          ctl = r[0];
          auto body = push(sc);
          for (size_t i = 0; i < st->names.size(); ++i)
            body->vars[st->names[i]] = std::make_shared<Value>(i < r.size() ? r[i] : Value());
          pop();
          Flow fl = exec_block(st->body, body);
          if (fl == F_BREAK) break;
          if (fl == F_RETURN || fl == F_GOTO) return fl;
        }
        return F_NORMAL;
      }
      case S_RETURN:
        ret = eval_list(st->exprs, s);
        return F_RETURN;
      case S_BREAK: return F_BREAK;
      case S_GOTO:
        go_label = st->names[0];
        return F_GOTO;
      case S_LABEL: return F_NORMAL;
    }
    return F_NORMAL;
  }
};

Value Interp::metamethod(const Value& v, const char* event) const {
  if (v.t == Value::Tab && v.tab->meta) return v.tab->meta->get(Value::string(event));
  if (v.t == Value::Str && string_meta) return string_meta->get(Value::string(event));
  return Value();
}

Value Interp::index(const Value& o0, const Value& k) {
  Value o = o0;
  for (int hop = 0; hop < 100; ++hop) {
    Value h;
    if (o.t == Value::Tab) {
      Value v = o.tab->get(k);
      if (v.t != Value::Nil) return v;
      h = metamethod(o, "__index");
      if (h.t == Value::Nil) return Value();
    } else if (o.t == Value::Str) {
      Value strlib = globals->get(Value::string("string"));
      return strlib.t == Value::Tab ? strlib.tab->get(k) : Value();
    } else {
      h = metamethod(o, "__index");
      if (h.t == Value::Nil) throw LuaError(std::string("attempt to index a ") + type_name(o) + " value");
    }
    if (h.t == Value::Fn) {
      Values r = call(h, {o, k});
      return r.empty() ? Value() : r[0];
    }
    o = h;
  }
  throw LuaError("'__index' chain too long; possible loop");
}

void Interp::setindex(const Value& o0, const Value& k, const Value& v) {
  Value o = o0;
  for (int hop = 0; hop < 100; ++hop) {
    Value h;
    if (o.t == Value::Tab) {
      if (o.tab->get(k).t != Value::Nil || (h = metamethod(o, "__newindex")).t == Value::Nil) {
        o.tab->set(k, v);
        return;
      }
    } else {
      h = metamethod(o, "__newindex");
      if (h.t == Value::Nil) throw LuaError(std::string("attempt to index a ") + type_name(o) + " value");
    }
    if (h.t == Value::Fn) {
      call(h, {o, k, v});
      return;
    }
    o = h;
  }
  throw LuaError("'__newindex' chain too long; possible loop");
}

std::string Interp::tostr(const Value& v) {
  Value h = v.t == Value::Tab ? metamethod(v, "__tostring") : Value();
  if (h.t != Value::Nil) {
    Values r = call(h, {v});
    if (r.empty() || r[0].t != Value::Str) throw LuaError("'__tostring' must return a string");
    return *r[0].s;
  }
  if (v.t == Value::Tab) {
    Value nm = metamethod(v, "__name");
    if (nm.t == Value::Str) {
      std::string t = tostring(v);
      return *nm.s + t.substr(t.find(':'));
    }
  }
  return tostring(v);
}

Values Interp::call(const Value& f0, Values args) {
  Value f = f0;
  if (f.t != Value::Fn) {
    Value h = metamethod(f, "__call");
    if (h.t != Value::Fn) throw LuaError(std::string("attempt to call a ") + type_name(f) + " value");
    args.insert(args.begin(), f);
    f = h;
  }
  if (++depth > 200) { --depth; throw LuaError("stack overflow"); }
  struct Guard { int& d; ~Guard() { --d; } } g{depth};
  if (f.fn->native) return f.fn->native(*this, args);
  const FuncBody& body = *f.fn->body;
  Exec ex(*this);
  auto sc = ex.push(f.fn->env);
  for (size_t i = 0; i < body.params.size(); ++i)
    sc->vars[body.params[i]] = std::make_shared<Value>(i < args.size() ? args[i] : Value());
  if (body.vararg) {
    sc->has_varargs = true;
    if (args.size() > body.params.size()) sc->varargs.assign(args.begin() + (long)body.params.size(), args.end());
  }
  Flow fl = ex.exec_block(body.block, sc);
  ex.pop();
  if (fl == F_GOTO) throw LuaError("no visible label '" + ex.go_label + "' for goto");
  return fl == F_RETURN ? ex.ret : Values{};
}

// ------------------------------------------------------------ stdlib ------
static Value arg_at(Values& a, size_t i) { return i < a.size() ? a[i] : Value(); }

static std::string check_str(Values& a, size_t i, const char* fn) {
  Value v = arg_at(a, i);
  if (v.t == Value::Str) return *v.s;
  if (v.is_num()) return tostring(v);
  throw LuaError(std::string("bad argument #") + std::to_string(i + 1) + " to '" + fn + "' (string expected, got " +
                 type_name(v) + ")");
}

static int64_t check_int(Values& a, size_t i, const char* fn) { return toint_strict(arg_at(a, i), fn); }

static double check_num(Values& a, size_t i, const char* fn) {
  Value n;
  if (!tonum(arg_at(a, i), &n))
    throw LuaError(std::string("bad argument #") + std::to_string(i + 1) + " to '" + fn + "' (number expected)");
  return n.as_double();
}

// ------------------------------------------------------------ patterns ----
// Lua 5.4 pattern matching (string.find / match / gmatch / gsub): single-character classes
// (. %a %c %d %g %l %p %s %u %w %x and their upper-case complements, %<punct> escapes, [sets]
// with ranges, classes and ^), quantifiers * + - ?, anchors ^ and $, captures ( ) and position
// captures (), back-references %1-%9, %bxy and the frontier %f[set].  A backtracking matcher over
// indices into the subject; recursion is bounded (kMaxDepth) so a pathological pattern fails
// with an error instead of exhausting the C stack.
namespace pat {

constexpr int kMaxCaptures = 32;
constexpr int kMaxDepth = 200;
constexpr long kOpen = -1;      // capture started, not closed
constexpr long kPosition = -2;  // () position capture
constexpr size_t kFail = std::string::npos;

struct Matcher {
  const std::string& src;
  const std::string& p;
  int level = 0;
  int depth = 0;
  size_t cap_start[kMaxCaptures];
  long cap_len[kMaxCaptures];

  Matcher(const std::string& s, const std::string& pattern) : src(s), p(pattern) {}

  static bool class_match(unsigned char c, unsigned char cl) {
    bool r;
    switch (tolower(cl)) {
      case 'a': r = isalpha(c); break;
      case 'c': r = iscntrl(c); break;
      case 'd': r = isdigit(c); break;
      case 'g': r = isgraph(c); break;
      case 'l': r = islower(c); break;
      case 'p': r = ispunct(c); break;
      case 's': r = isspace(c); break;
      case 'u': r = isupper(c); break;
      case 'w': r = isalnum(c); break;
      case 'x': r = isxdigit(c); break;
      default: return cl == c;  // escaped literal (%. %% %[ ...)
    }
    return isupper(cl) ? !r : r;
  }

  // index just past the single-character class starting at pi
  size_t class_end(size_t pi) const {
    const size_t n = p.size();
    const char c = p[pi++];
    if (c == '%') {
      if (pi >= n) throw LuaError("malformed pattern (ends with '%')");
      return pi + 1;
    }
    if (c == '[') {
      if (pi < n && p[pi] == '^') ++pi;
      const size_t first = pi;
      for (;;) {  // a ']' right after '[' or '[^' is a literal member
        if (pi >= n) throw LuaError("malformed pattern (missing ']')");
        if (p[pi] == ']' && pi != first) return pi + 1;
        if (p[pi] == '%') {
          if (pi + 1 >= n) throw LuaError("malformed pattern (missing ']')");
          pi += 2;
        } else {
          ++pi;
        }
      }
    }
    return pi;
  }

  // [set] at p[open] .. p[close] (close = index of the ']')
  bool set_match(unsigned char c, size_t open, size_t close) const {
    size_t i = open + 1;
    bool neg = false;
    if (p[i] == '^') {
      neg = true;
      ++i;
    }
    while (i < close) {  // class_end put close past a leading literal ']'
      if (p[i] == '%' && i + 1 < close) {
        if (class_match(c, (unsigned char)p[i + 1])) return !neg;
        i += 2;
      } else if (i + 2 < close && p[i + 1] == '-') {
        if ((unsigned char)p[i] <= c && c <= (unsigned char)p[i + 2]) return !neg;
        i += 3;
      } else {
        if ((unsigned char)p[i] == c) return !neg;
        ++i;
      }
    }
    return neg;
  }

  bool single(size_t s, size_t pi, size_t ep) const {
    if (s >= src.size()) return false;
    const unsigned char c = (unsigned char)src[s];
    switch (p[pi]) {
      case '.': return true;
      case '%': return class_match(c, (unsigned char)p[pi + 1]);
      case '[': return set_match(c, pi, ep - 1);
      default: return (unsigned char)p[pi] == c;
    }
  }

  size_t max_expand(size_t s, size_t pi, size_t ep) {
    size_t i = 0;
    while (single(s + i, pi, ep)) ++i;
    for (;;) {  // longest first, then give back one at a time
      const size_t r = match(s + i, ep + 1);
      if (r != kFail) return r;
      if (i == 0) return kFail;
      --i;
    }
  }

  size_t min_expand(size_t s, size_t pi, size_t ep) {
    for (;;) {
      const size_t r = match(s, ep + 1);
      if (r != kFail) return r;
      if (!single(s, pi, ep)) return kFail;
      ++s;
    }
  }

  size_t start_capture(size_t s, size_t pi, long what) {
    if (level >= kMaxCaptures) throw LuaError("too many captures");
    cap_start[level] = s;
    cap_len[level] = what;
    ++level;
    const size_t r = match(s, pi);
    if (r == kFail) --level;
    return r;
  }

  size_t end_capture(size_t s, size_t pi) {
    int l = -1;
    for (int i = level - 1; i >= 0; --i)
      if (cap_len[i] == kOpen) {
        l = i;
        break;
      }
    if (l < 0) throw LuaError("invalid pattern capture");
    cap_len[l] = (long)(s - cap_start[l]);
    const size_t r = match(s, pi);
    if (r == kFail) cap_len[l] = kOpen;
    return r;
  }

  size_t back_reference(size_t s, char d) const {
    const int l = d - '1';
    if (l < 0 || l >= level || cap_len[l] == kOpen) throw LuaError(std::string("invalid capture index %") + d);
    const size_t len = cap_len[l] == kPosition ? 0 : (size_t)cap_len[l];
    if (src.size() - s >= len && src.compare(cap_start[l], len, src, s, len) == 0) return s + len;
    return kFail;
  }

  size_t balance(size_t s, size_t pi) const {
    if (pi + 1 >= p.size()) throw LuaError("malformed pattern (missing arguments to '%b')");
    if (s >= src.size() || src[s] != p[pi]) return kFail;
    const char open = p[pi], close = p[pi + 1];
    int depth_ = 1;
    for (size_t i = s + 1; i < src.size(); ++i) {
      if (src[i] == close) {
        if (--depth_ == 0) return i + 1;
      } else if (src[i] == open) {
        ++depth_;
      }
    }
    return kFail;
  }

  // end of the match of p[pi..] at src[s..], or kFail
  size_t match(size_t s, size_t pi) {
    if (++depth > kMaxDepth) throw LuaError("pattern too complex");
    struct Guard {
      int& d;
      ~Guard() { --d; }
    } guard{depth};
    const size_t n = p.size();
    for (;;) {
      if (pi == n) return s;
      const char pc = p[pi];
      if (pc == '(') {
        if (pi + 1 < n && p[pi + 1] == ')') return start_capture(s, pi + 2, kPosition);
        return start_capture(s, pi + 1, kOpen);
      }
      if (pc == ')') return end_capture(s, pi + 1);
      if (pc == '$' && pi + 1 == n) return s == src.size() ? s : kFail;
      if (pc == '%' && pi + 1 < n) {
        const char nx = p[pi + 1];
        if (nx == 'b') {
          s = balance(s, pi + 2);
          if (s == kFail) return kFail;
          pi += 4;
          continue;
        }
        if (nx == 'f') {
          pi += 2;
          if (pi >= n || p[pi] != '[') throw LuaError("missing '[' after '%f' in pattern");
          const size_t ep = class_end(pi);
          const unsigned char prev = s == 0 ? 0 : (unsigned char)src[s - 1];
          const unsigned char cur = s < src.size() ? (unsigned char)src[s] : 0;
          if (set_match(prev, pi, ep - 1) || !set_match(cur, pi, ep - 1)) return kFail;
          pi = ep;
          continue;
        }
        if (isdigit((unsigned char)nx)) {
          s = back_reference(s, nx);
          if (s == kFail) return kFail;
          pi += 2;
          continue;
        }
      }
      const size_t ep = class_end(pi);
      const char q = ep < n ? p[ep] : 0;
      if (q == '?') {
        if (single(s, pi, ep)) {
          const size_t r = match(s + 1, ep + 1);
          if (r != kFail) return r;
        }
        pi = ep + 1;
        continue;
      }
      if (q == '+') return single(s, pi, ep) ? max_expand(s + 1, pi, ep) : kFail;
      if (q == '*') return max_expand(s, pi, ep);
      if (q == '-') return min_expand(s, pi, ep);
      if (!single(s, pi, ep)) return kFail;
      ++s;
      pi = ep;
    }
  }

  Value capture(int i, size_t s, size_t e) const {
    if (i >= level) {
      if (i == 0) return Value::string(src.substr(s, e - s));  // no captures: the whole match
      throw LuaError("invalid capture index %" + std::to_string(i + 1));
    }
    if (cap_len[i] == kOpen) throw LuaError("unfinished capture");
    if (cap_len[i] == kPosition) return Value::integer((int64_t)cap_start[i] + 1);
    return Value::string(src.substr(cap_start[i], (size_t)cap_len[i]));
  }

  Values captures(size_t s, size_t e, bool whole_if_none) const {
    Values r;
    const int nc = (level == 0 && whole_if_none) ? 1 : level;
    for (int i = 0; i < nc; ++i) r.push_back(capture(i, s, e));
    return r;
  }

  // try at every start position from `init` (0-based); returns the start or kFail, *end = match end
  size_t search(size_t init, size_t* end) {
    const bool anchor = !p.empty() && p[0] == '^';
    const size_t p0 = anchor ? 1 : 0;
    for (size_t s = init;; ++s) {
      level = 0;
      depth = 0;
      const size_t e = match(s, p0);
      if (e != kFail) {
        *end = e;
        return s;
      }
      if (anchor || s >= src.size()) return kFail;
    }
  }
};

static bool has_specials(const std::string& p) { return p.find_first_of("^$*+?.([%-") != std::string::npos; }

// string.find / string.match
static Values find_aux(Values& a, bool find, const char* fn) {
  const std::string s = check_str(a, 0, fn), pt = check_str(a, 1, fn);
  int64_t init = a.size() > 2 && a[2].t != Value::Nil ? check_int(a, 2, fn) : 1;
  const int64_t len = (int64_t)s.size();
  if (init < 0) init = len + init + 1;
  if (init < 1) init = 1;
  if (init > len + 1) return Values{Value()};
  const bool plain = a.size() > 3 && a[3].truthy();
  if (find && (plain || !has_specials(pt))) {
    const size_t pos = s.find(pt, (size_t)init - 1);
    if (pos == std::string::npos) return Values{Value()};
    return Values{Value::integer((int64_t)pos + 1), Value::integer((int64_t)(pos + pt.size()))};
  }
  Matcher m(s, pt);
  size_t e = 0;
  const size_t st = m.search((size_t)init - 1, &e);
  if (st == kFail) return Values{Value()};
  if (!find) return m.captures(st, e, true);
  Values r{Value::integer((int64_t)st + 1), Value::integer((int64_t)e)};
  Values c = m.captures(st, e, false);
  r.insert(r.end(), c.begin(), c.end());
  return r;
}

}  // namespace pat

// ------------------------------------------------------------ coroutines --
// Each coroutine runs its function on a thread of its own; resume and yield hand a single
// "turn" back and forth under a mutex, so exactly one thread runs Lua code at any time and the
// tree-walking evaluator needs no changes: a yield inside nested Lua calls, pcall, metamethods
// or a native callback simply blocks that thread's C++ stack until the next resume.  A
// suspended coroutine that is collected or closed is unwound with CoKill (not a LuaError, so
// pcall inside it cannot catch it) and joined.
struct CoKill {};

struct Coroutine : std::enable_shared_from_this<Coroutine> {
  enum Status { Suspended, Running, Normal, Dead };
  Value fn;
  Status st = Suspended;
  Interp* I = nullptr;
  Heap* heap = nullptr;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  bool co_turn = false;  // true: the coroutine's thread runs; false: its resumer runs
  bool killed = false;
  bool failed = false;
  int depth = 0;         // interpreter call depth of the coroutine's own stack
  Values transfer;       // resume arguments in, yield / return values out

  ~Coroutine() { kill(); }

  void kill() {
    if (!th.joinable()) return;
    {
      std::unique_lock<std::mutex> l(mu);
      if (st != Dead) {
        killed = true;
        co_turn = true;
        cv.notify_all();
        cv.wait(l, [&] { return !co_turn; });
      }
    }
    th.join();
    st = Dead;
  }
};

static thread_local Coroutine* t_co = nullptr;  // the coroutine this thread runs (null: main)

static void co_body(Coroutine* c) {
  t_heap = c->heap;
  t_co = c;
  {
    std::unique_lock<std::mutex> l(c->mu);
    c->cv.wait(l, [&] { return c->co_turn; });
  }
  Values out;
  bool failed = false;
  if (!c->killed) {
    try {
      Values args = std::move(c->transfer);
      out = c->I->call(c->fn, std::move(args));
    } catch (LuaError& e) {
      failed = true;
      out = Values{e.value};
    } catch (CoKill&) {
    } catch (std::exception& e) {
      failed = true;
      out = Values{Value::string(e.what())};
    }
  }
  std::lock_guard<std::mutex> l(c->mu);
  c->transfer = std::move(out);
  c->failed = failed;
  c->st = Coroutine::Dead;
  c->co_turn = false;
  c->cv.notify_all();
}

static Values co_resume(Interp& I, const std::shared_ptr<Coroutine>& c, Values args) {
  if (c->st == Coroutine::Dead) return Values{Value::boolean(false), Value::string("cannot resume dead coroutine")};
  if (c->st != Coroutine::Suspended)
    return Values{Value::boolean(false), Value::string("cannot resume non-suspended coroutine")};
  Coroutine* prev = t_co;
  if (prev) prev->st = Coroutine::Normal;
  const int saved_depth = I.depth;
  I.depth = c->depth;
  {
    std::unique_lock<std::mutex> l(c->mu);
    c->transfer = std::move(args);
    c->st = Coroutine::Running;
    if (!c->th.joinable()) c->th = std::thread(co_body, c.get());
    c->co_turn = true;
    c->cv.notify_all();
    c->cv.wait(l, [&] { return !c->co_turn; });
  }
  c->depth = I.depth;
  I.depth = saved_depth;
  if (prev) prev->st = Coroutine::Running;
  Values r = std::move(c->transfer);
  c->transfer.clear();
  if (c->failed) {
    c->failed = false;
    r.insert(r.begin(), Value::boolean(false));
    return r;
  }
  r.insert(r.begin(), Value::boolean(true));
  return r;
}

static Values co_yield(Values vals) {
  Coroutine* c = t_co;
  if (!c) throw LuaError("attempt to yield from outside a coroutine");
  std::unique_lock<std::mutex> l(c->mu);
  c->transfer = std::move(vals);
  c->st = Coroutine::Suspended;
  c->co_turn = false;
  c->cv.notify_all();
  c->cv.wait(l, [&] { return c->co_turn; });
  if (c->killed) throw CoKill{};
  return std::move(c->transfer);
}

static std::string lua_format(Values& a) {
  const std::string fmt = check_str(a, 0, "format");
  std::string out;
  size_t ai = 1;
  for (size_t i = 0; i < fmt.size(); ++i) {
    if (fmt[i] != '%') { out += fmt[i]; continue; }
    if (++i >= fmt.size()) throw LuaError("invalid conversion '%' to 'format'");
    if (fmt[i] == '%') { out += '%'; continue; }
    std::string spec = "%";
    while (i < fmt.size() && strchr("-+ #0123456789.", fmt[i])) spec += fmt[i++];
    if (i >= fmt.size()) throw LuaError("invalid conversion to 'format'");
    const char c = fmt[i];
    char buf[512];
    switch (c) {
      case 'd': case 'i': {
        spec += "lld";
        snprintf(buf, sizeof buf, spec.c_str(), (long long)check_int(a, ai++, "format"));
        out += buf;
        break;
      }
      case 'u': case 'x': case 'X': case 'o': case 'c': {
        if (c == 'c') { out += (char)check_int(a, ai++, "format"); break; }
        spec += "ll";
        spec += c;
        snprintf(buf, sizeof buf, spec.c_str(), (unsigned long long)check_int(a, ai++, "format"));
        out += buf;
        break;
      }
      case 'f': case 'F': case 'e': case 'E': case 'g': case 'G': case 'a': case 'A': {
        spec += c;
        snprintf(buf, sizeof buf, spec.c_str(), check_num(a, ai++, "format"));
        out += buf;
        break;
      }
      case 's': {
        Value v = arg_at(a, ai++);
        std::string sv = tostring(v);
        spec += 's';
        if (spec == "%s") out += sv;
        else { snprintf(buf, sizeof buf, spec.c_str(), sv.c_str()); out += buf; }
        break;
      }
      case 'q': {
        Value v = arg_at(a, ai++);
        if (v.t != Value::Str) {
          // integers as themselves, floats in hex (%a) so they read back exactly (lstrlib.c quotefloat)
          if (v.t == Value::Num) {
            if (v.n == (double)(int64_t)v.n) snprintf(buf, sizeof buf, "%lld.0", (long long)v.n);
            else snprintf(buf, sizeof buf, "%a", v.n);
            out += buf;
          } else {
            out += tostring(v);
          }
          break;
        }
        out += '"';
        const std::string& sv = *v.s;
        for (size_t q = 0; q < sv.size(); ++q) {
          const unsigned char ch = (unsigned char)sv[q];
          if (ch == '"' || ch == '\\') { out += '\\'; out += (char)ch; }
          else if (ch == '\n') out += "\\\n";  // backslash-newline, as Lua 5.4
          else if (ch == '\r') out += "\\r";
          else if (ch == 0) out += (q + 1 < sv.size() && isdigit((unsigned char)sv[q + 1])) ? "\\000" : "\\0";
          else if (ch < 32 || ch == 127) {
            // a following digit would extend the escape: pad to three digits then (lstrlib.c addquoted)
            snprintf(buf, sizeof buf, (q + 1 < sv.size() && isdigit((unsigned char)sv[q + 1])) ? "\\%03d" : "\\%d", ch);
            out += buf;
          }
          else out += (char)ch;
        }
        out += '"';
        break;
      }
      default: throw LuaError(std::string("invalid conversion '%") + c + "' to 'format'");
    }
  }
  return out;
}

static void reg(const std::shared_ptr<Table>& t, const char* name, Native f) {
  t->set(Value::string(name), make_native(name, std::move(f)));
}

Interp::Interp() {
  heap = new Heap;
  prev_heap = t_heap;
  t_heap = heap;
  globals = std::make_shared<Table>();
  root = std::make_shared<Scope>();
  out = [](const std::string& s) { fwrite(s.data(), 1, s.size(), stdout); };
  auto G = globals;
  G->set(Value::string("_G"), Value::table(G));
  G->set(Value::string("_VERSION"), Value::string("Lua 5.4 (splinterctl minilua)"));
  reg(G, "print", [](Interp& I, Values& a) {
    std::string line;
    for (size_t i = 0; i < a.size(); ++i) line += (i ? "\t" : "") + I.tostr(a[i]);
    line += '\n';
    I.out(line);
    return Values{};
  });
  reg(G, "type", [](Interp&, Values& a) {
    if (a.empty()) throw LuaError("bad argument #1 to 'type' (value expected)");
    return Values{Value::string(type_name(a[0]))};
  });
  reg(G, "tostring", [](Interp& I, Values& a) { return Values{Value::string(I.tostr(arg_at(a, 0)))}; });
  reg(G, "setmetatable", [](Interp& I, Values& a) {
    Value t = arg_at(a, 0), m = arg_at(a, 1);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'setmetatable' (table expected)");
    if (m.t != Value::Nil && m.t != Value::Tab)
      throw LuaError("bad argument #2 to 'setmetatable' (nil or table expected)");
    if (I.metamethod(t, "__metatable").t != Value::Nil) throw LuaError("cannot change a protected metatable");
    t.tab->meta = m.t == Value::Tab ? m.tab : nullptr;
    // marked for finalization when the metatable has __gc at this point (a field added later does not count)
    if (m.t == Value::Tab && m.tab->get(Value::string("__gc")).t != Value::Nil &&
        std::find(I.finalizers.begin(), I.finalizers.end(), t.tab) == I.finalizers.end())
      I.finalizers.push_back(t.tab);
    return Values{t};
  });
  reg(G, "collectgarbage", [](Interp& I, Values& a) -> Values {
    const std::string opt = a.empty() || a[0].t == Value::Nil ? "collect" : check_str(a, 0, "collectgarbage");
    if (opt == "collect" || opt == "step") {
      I.run_finalizers(false);
      return Values{opt == "step" ? Value::boolean(true) : Value::integer(0)};
    }
    if (opt == "count") {  // KB in use, estimated from the live objects (tables and scopes)
      const double kb = I.heap ? (double)(I.heap->tables.size() * 96 + I.heap->scopes.size() * 112) / 1024.0 : 0.0;
      return Values{Value::number(kb)};
    }
    if (opt == "isrunning") return Values{Value::boolean(true)};
    if (opt == "incremental" || opt == "generational") return Values{Value::string("incremental")};
    if (opt == "stop" || opt == "restart" || opt == "setpause" || opt == "setstepmul") return Values{Value::integer(0)};
    throw LuaError("bad argument #1 to 'collectgarbage' (invalid option '" + opt + "')");
  });
  reg(G, "getmetatable", [](Interp& I, Values& a) {
    Value v = arg_at(a, 0);
    std::shared_ptr<Table> m = v.t == Value::Tab ? v.tab->meta : v.t == Value::Str ? I.string_meta : nullptr;
    if (!m) return Values{Value()};
    Value prot = m->get(Value::string("__metatable"));
    return Values{prot.t != Value::Nil ? prot : Value::table(m)};
  });
  reg(G, "tonumber", [](Interp&, Values& a) {
    Value v = arg_at(a, 0), n;
    if (a.size() > 1 && arg_at(a, 1).t != Value::Nil) {
      const int64_t base = check_int(a, 1, "tonumber");
      char* end = nullptr;
      std::string s = check_str(a, 0, "tonumber");
      long long r = strtoll(s.c_str(), &end, (int)base);
      return Values{*end == 0 && !s.empty() ? Value::integer(r) : Value()};
    }
    return Values{tonum(v, &n) ? n : Value()};
  });
  reg(G, "rawequal", [](Interp&, Values& a) { return Values{Value::boolean(raw_equal(arg_at(a, 0), arg_at(a, 1)))}; });
  reg(G, "rawget", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'rawget' (table expected)");
    return Values{t.tab->get(arg_at(a, 1))};
  });
  reg(G, "rawset", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'rawset' (table expected)");
    t.tab->set(arg_at(a, 1), arg_at(a, 2));
    return Values{t};
  });
  reg(G, "rawlen", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t == Value::Tab) return Values{Value::integer(t.tab->length())};
    if (t.t == Value::Str) return Values{Value::integer((int64_t)t.s->size())};
    throw LuaError("table or string expected");
  });
  auto next = make_native("next", [](Interp&, Values& a) {
    Value t = arg_at(a, 0), k = arg_at(a, 1);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'next' (table expected)");
    auto& T = *t.tab;
    size_t i = 0;
    if (k.t != Value::Nil) {
      auto it = T.index.find(norm_key(k));
      if (it == T.index.end()) throw LuaError("invalid key to 'next'");
      i = it->second + 1;
    }
    for (; i < T.entries.size(); ++i)
      if (T.entries[i].second.t != Value::Nil) return Values{T.entries[i].first, T.entries[i].second};
    return Values{Value()};
  });
  G->set(Value::string("next"), next);
  reg(G, "pairs", [next](Interp& I, Values& a) {
    Value h = I.metamethod(arg_at(a, 0), "__pairs");
    if (h.t != Value::Nil) {
      Values r = I.call(h, {a[0]});
      r.resize(3);
      return r;
    }
    if (arg_at(a, 0).t != Value::Tab) throw LuaError("bad argument #1 to 'pairs' (table expected)");
    return Values{next, a[0], Value()};
  });
  auto ipairs_iter = make_native("ipairs_iter", [](Interp& I, Values& a) {
    Value t = arg_at(a, 0);
    const int64_t i = arg_at(a, 1).i + 1;
    Value v = I.index(t, Value::integer(i));  // honours __index, as lua_geti does
    if (v.t == Value::Nil) return Values{Value()};
    return Values{Value::integer(i), v};
  });
  reg(G, "ipairs", [ipairs_iter](Interp&, Values& a) {
    if (arg_at(a, 0).t != Value::Tab) throw LuaError("bad argument #1 to 'ipairs' (table expected)");
    return Values{ipairs_iter, a[0], Value::integer(0)};
  });
  reg(G, "select", [](Interp&, Values& a) {
    Value n = arg_at(a, 0);
    if (n.t == Value::Str && *n.s == "#") return Values{Value::integer((int64_t)a.size() - 1)};
    int64_t i = check_int(a, 0, "select");
    if (i < 0) i = (int64_t)a.size() + i;
    if (i < 1) throw LuaError("bad argument #1 to 'select' (index out of range)");
    if ((size_t)i >= a.size()) return Values{};
    return Values(a.begin() + i, a.end());
  });
  reg(G, "error", [](Interp& I, Values& a) -> Values {
    Value v = arg_at(a, 0);
    const int64_t level = a.size() > 1 ? toint_strict(a[1], "error") : 1;
    if (v.t == Value::Str && level > 0) v = Value::string(I.chunk + ":" + std::to_string(I.line) + ": " + *v.s);
    throw LuaError(v, v.t == Value::Str ? *v.s : tostring(v));
  });
  reg(G, "assert", [](Interp&, Values& a) -> Values {
    if (!arg_at(a, 0).truthy()) {
      Value m = a.size() > 1 ? a[1] : Value::string("assertion failed!");
      throw LuaError(m, tostring(m));
    }
    return a;
  });
  reg(G, "pcall", [](Interp& I, Values& a) {
    if (a.empty()) throw LuaError("bad argument #1 to 'pcall' (value expected)");
    Value f = a[0];
    Values rest(a.begin() + 1, a.end());
    const int d = I.depth;
    try {
      Values r = I.call(f, rest);
      r.insert(r.begin(), Value::boolean(true));
      return r;
    } catch (LuaError& e) {
      I.depth = d;
      return Values{Value::boolean(false), e.value};
    }
  });
  auto unpack = make_native("unpack", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'unpack' (table expected)");
    int64_t i = a.size() > 1 && a[1].t != Value::Nil ? check_int(a, 1, "unpack") : 1;
    int64_t j = a.size() > 2 && a[2].t != Value::Nil ? check_int(a, 2, "unpack") : t.tab->length();
    Values r;
    for (; i <= j; ++i) r.push_back(t.tab->get(Value::integer(i)));
    return r;
  });
  G->set(Value::string("unpack"), unpack);
  reg(G, "require", [](Interp& I, Values& a) {
    const std::string n = check_str(a, 0, "require");
    auto it = I.modules.find(n);
    if (it == I.modules.end()) throw LuaError("module '" + n + "' not found");
    return Values{it->second};
  });

  // coroutine
  auto C = std::make_shared<Table>();
  G->set(Value::string("coroutine"), Value::table(C));
  auto check_co = [](Values& a, const char* fn) {
    Value v = arg_at(a, 0);
    if (v.t != Value::Co) throw LuaError(std::string("bad argument #1 to '") + fn + "' (coroutine expected)");
    return v.co;
  };
  reg(C, "create", [](Interp& I, Values& a) {
    Value f = arg_at(a, 0);
    if (f.t != Value::Fn) throw LuaError("bad argument #1 to 'create' (function expected)");
    auto c = std::make_shared<Coroutine>();
    c->fn = f;
    c->I = &I;
    c->heap = I.heap;
    return Values{Value::thread(c)};
  });
  reg(C, "resume", [check_co](Interp& I, Values& a) {
    auto c = check_co(a, "resume");
    return co_resume(I, c, Values(a.begin() + 1, a.end()));
  });
  reg(C, "yield", [](Interp&, Values& a) { return co_yield(a); });
  reg(C, "status", [check_co](Interp&, Values& a) {
    static const char* names[] = {"suspended", "running", "normal", "dead"};
    return Values{Value::string(names[check_co(a, "status")->st])};
  });
  reg(C, "running", [](Interp&, Values&) {
    if (!t_co) return Values{Value(), Value::boolean(true)};  // main: no thread object in minilua
    return Values{Value::thread(t_co->shared_from_this()), Value::boolean(false)};
  });
  reg(C, "isyieldable", [](Interp&, Values&) { return Values{Value::boolean(t_co != nullptr)}; });
  reg(C, "close", [check_co](Interp&, Values& a) {
    auto c = check_co(a, "close");
    if (c->st == Coroutine::Running || c->st == Coroutine::Normal)
      throw LuaError("cannot close a running coroutine");
    c->kill();
    c->st = Coroutine::Dead;
    return Values{Value::boolean(true)};
  });
  reg(C, "wrap", [](Interp& I, Values& a) {
    Value f = arg_at(a, 0);
    if (f.t != Value::Fn) throw LuaError("bad argument #1 to 'wrap' (function expected)");
    auto c = std::make_shared<Coroutine>();
    c->fn = f;
    c->I = &I;
    c->heap = I.heap;
    return Values{make_native("wrap", [c](Interp& In, Values& args) {
      Values r = co_resume(In, c, args);
      if (!r[0].truthy()) {
        Value e = r.size() > 1 ? r[1] : Value();
        throw LuaError(e, e.t == Value::Str ? *e.s : tostring(e));
      }
      r.erase(r.begin());
      return r;
    })};
  });

  // string
  auto S = std::make_shared<Table>();
  G->set(Value::string("string"), Value::table(S));
  string_meta = std::make_shared<Table>();
  string_meta->set(Value::string("__index"), Value::table(S));
  reg(S, "format", [](Interp&, Values& a) { return Values{Value::string(lua_format(a))}; });
  reg(S, "len", [](Interp&, Values& a) { return Values{Value::integer((int64_t)check_str(a, 0, "len").size())}; });
  reg(S, "upper", [](Interp&, Values& a) {
    std::string s = check_str(a, 0, "upper");
    for (auto& c : s) c = (char)toupper((unsigned char)c);
    return Values{Value::string(s)};
  });
  reg(S, "lower", [](Interp&, Values& a) {
    std::string s = check_str(a, 0, "lower");
    for (auto& c : s) c = (char)tolower((unsigned char)c);
    return Values{Value::string(s)};
  });
  reg(S, "reverse", [](Interp&, Values& a) {
    std::string s = check_str(a, 0, "reverse");
    std::reverse(s.begin(), s.end());
    return Values{Value::string(s)};
  });
  reg(S, "rep", [](Interp&, Values& a) {
    std::string s = check_str(a, 0, "rep"), sep = a.size() > 2 ? check_str(a, 2, "rep") : "";
    int64_t n = check_int(a, 1, "rep");
    std::string out;
    for (int64_t i = 0; i < n; ++i) { if (i) out += sep; out += s; }
    return Values{Value::string(out)};
  });
  auto sub_idx = [](int64_t i, int64_t len) -> int64_t {
    if (i < 0) i = len + i + 1;
    return i;
  };
  reg(S, "sub", [sub_idx](Interp&, Values& a) {
    std::string s = check_str(a, 0, "sub");
    const int64_t len = (int64_t)s.size();
    int64_t i = a.size() > 1 ? sub_idx(check_int(a, 1, "sub"), len) : 1;
    int64_t j = a.size() > 2 && a[2].t != Value::Nil ? sub_idx(check_int(a, 2, "sub"), len) : len;
    if (i < 1) i = 1;
    if (j > len) j = len;
    if (i > j) return Values{Value::string("")};
    return Values{Value::string(s.substr((size_t)(i - 1), (size_t)(j - i + 1)))};
  });
  reg(S, "byte", [sub_idx](Interp&, Values& a) {
    std::string s = check_str(a, 0, "byte");
    const int64_t len = (int64_t)s.size();
    int64_t i = a.size() > 1 ? sub_idx(check_int(a, 1, "byte"), len) : 1;
    int64_t j = a.size() > 2 ? sub_idx(check_int(a, 2, "byte"), len) : i;
    Values r;
    for (int64_t k = std::max<int64_t>(i, 1); k <= std::min(j, len); ++k)
      r.push_back(Value::integer((unsigned char)s[(size_t)k - 1]));
    return r;
  });
  reg(S, "char", [](Interp&, Values& a) {
    std::string s;
    for (size_t i = 0; i < a.size(); ++i) s += (char)check_int(a, i, "char");
    return Values{Value::string(s)};
  });
  reg(S, "find", [](Interp&, Values& a) { return pat::find_aux(a, true, "find"); });
  reg(S, "match", [](Interp&, Values& a) { return pat::find_aux(a, false, "match"); });
  reg(S, "gmatch", [](Interp&, Values& a) {
    struct State {
      std::string src, p;
      size_t pos = 0, last = pat::kFail;
    };
    auto st = std::make_shared<State>();
    st->src = check_str(a, 0, "gmatch");
    st->p = check_str(a, 1, "gmatch");
    int64_t init = a.size() > 2 && a[2].t != Value::Nil ? check_int(a, 2, "gmatch") : 1;
    const int64_t len = (int64_t)st->src.size();
    if (init < 0) init = len + init + 1;
    if (init < 1) init = 1;
    st->pos = (size_t)std::min<int64_t>(init - 1, len + 1);
    return Values{make_native("gmatch_iter", [st](Interp&, Values&) {
      pat::Matcher m(st->src, st->p);  // '^' is not an anchor in gmatch (Lua 5.4): matched literally
      for (size_t s = st->pos; s <= st->src.size(); ++s) {
        m.level = 0;
        m.depth = 0;
        const size_t e = m.match(s, 0);
        if (e != pat::kFail && e != st->last) {
          st->pos = st->last = e;
          return m.captures(s, e, true);
        }
      }
      st->pos = st->src.size() + 1;
      return Values{Value()};
    })};
  });
  reg(S, "gsub", [](Interp& I, Values& a) {
    const std::string src = check_str(a, 0, "gsub"), p = check_str(a, 1, "gsub");
    const Value repl = arg_at(a, 2);
    if (repl.t != Value::Str && !repl.is_num() && repl.t != Value::Tab && repl.t != Value::Fn)
      throw LuaError(std::string("bad argument #3 to 'gsub' (string/function/table expected, got ") +
                     type_name(repl) + ")");
    const int64_t max_n = a.size() > 3 && a[3].t != Value::Nil ? check_int(a, 3, "gsub") : INT64_MAX;
    const std::string rs = repl.t == Value::Str || repl.is_num() ? check_str(a, 2, "gsub") : "";
    const bool anchor = !p.empty() && p[0] == '^';
    pat::Matcher m(src, p);
    std::string out;
    size_t s = 0, last = pat::kFail;
    int64_t n = 0;
    while (n < max_n) {
      m.level = 0;
      m.depth = 0;
      const size_t e = m.match(s, anchor ? 1 : 0);
      if (e != pat::kFail && e != last) {
        ++n;
        Value r;
        if (repl.t == Value::Str || repl.is_num()) {
          std::string piece;
          for (size_t i = 0; i < rs.size(); ++i) {
            if (rs[i] != '%') { piece += rs[i]; continue; }
            if (++i >= rs.size()) throw LuaError("invalid use of '%' in replacement string");
            const char d = rs[i];
            if (d == '%') piece += '%';
            else if (d == '0') piece += src.substr(s, e - s);
            else if (isdigit((unsigned char)d)) piece += I.tostr(m.capture(d - '1', s, e));
            else throw LuaError("invalid use of '%' in replacement string");
          }
          r = Value::string(piece);
        } else {
          Value c0 = m.capture(0, s, e);
          if (repl.t == Value::Tab) {
            r = I.index(repl, c0);
          } else {
            Values rv = I.call(repl, m.captures(s, e, true));
            r = rv.empty() ? Value() : rv[0];
          }
        }
        if (!r.truthy()) out += src.substr(s, e - s);  // false / nil: keep the original match
        else if (r.t == Value::Str || r.is_num()) out += r.t == Value::Str ? *r.s : tostring(r);
        else throw LuaError(std::string("invalid replacement value (a ") + type_name(r) + ")");
        s = last = e;
      } else if (s < src.size()) {
        out += src[s++];
      } else {
        break;
      }
      if (anchor) break;
    }
    if (s < src.size()) out += src.substr(s);
    return Values{Value::string(out), Value::integer(n)};
  });

  // table
  auto T = std::make_shared<Table>();
  G->set(Value::string("table"), Value::table(T));
  T->set(Value::string("unpack"), unpack);
  reg(T, "insert", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'insert' (table expected)");
    const int64_t n = t.tab->length();
    if (a.size() == 2) {
      t.tab->set(Value::integer(n + 1), a[1]);
    } else if (a.size() == 3) {
      int64_t pos = check_int(a, 1, "insert");
      if (pos < 1 || pos > n + 1) throw LuaError("bad argument #2 to 'insert' (position out of bounds)");
      for (int64_t i = n; i >= pos; --i) t.tab->set(Value::integer(i + 1), t.tab->get(Value::integer(i)));
      t.tab->set(Value::integer(pos), a[2]);
    } else {
      throw LuaError("wrong number of arguments to 'insert'");
    }
    return Values{};
  });
  reg(T, "remove", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'remove' (table expected)");
    const int64_t n = t.tab->length();
    int64_t pos = a.size() > 1 ? check_int(a, 1, "remove") : n;
    if (n == 0) return Values{Value()};
    Value v = t.tab->get(Value::integer(pos));
    for (int64_t i = pos; i < n; ++i) t.tab->set(Value::integer(i), t.tab->get(Value::integer(i + 1)));
    t.tab->set(Value::integer(n), Value());
    return Values{v};
  });
  reg(T, "concat", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'concat' (table expected)");
    std::string sep = a.size() > 1 && a[1].t != Value::Nil ? check_str(a, 1, "concat") : "";
    int64_t i = a.size() > 2 ? check_int(a, 2, "concat") : 1, j = a.size() > 3 ? check_int(a, 3, "concat") : t.tab->length();
    std::string out;
    for (int64_t k = i; k <= j; ++k) {
      Value v = t.tab->get(Value::integer(k));
      if (v.t != Value::Str && !v.is_num()) throw LuaError("invalid value (at index " + std::to_string(k) + ") in table for 'concat'");
      if (k > i) out += sep;
      out += tostring(v);
    }
    return Values{Value::string(out)};
  });

  // math
  auto M = std::make_shared<Table>();
  G->set(Value::string("math"), Value::table(M));
  M->set(Value::string("pi"), Value::number(M_PI));
  M->set(Value::string("huge"), Value::number(HUGE_VAL));
  M->set(Value::string("maxinteger"), Value::integer(INT64_MAX));
  M->set(Value::string("mininteger"), Value::integer(INT64_MIN));
  auto int_or_float = [](double d) {
    int64_t i;
    return float_is_int(d, &i) ? Value::integer(i) : Value::number(d);
  };
  reg(M, "floor", [int_or_float](Interp&, Values& a) {
    Value v = arg_at(a, 0);
    if (v.t == Value::Int) return Values{v};
    return Values{int_or_float(std::floor(check_num(a, 0, "floor")))};
  });
  reg(M, "ceil", [int_or_float](Interp&, Values& a) {
    Value v = arg_at(a, 0);
    if (v.t == Value::Int) return Values{v};
    return Values{int_or_float(std::ceil(check_num(a, 0, "ceil")))};
  });
  reg(M, "abs", [](Interp&, Values& a) {
    Value v = arg_at(a, 0);
    if (v.t == Value::Int) return Values{Value::integer(v.i < 0 ? -v.i : v.i)};
    return Values{Value::number(std::fabs(check_num(a, 0, "abs")))};
  });
  reg(M, "sqrt", [](Interp&, Values& a) { return Values{Value::number(std::sqrt(check_num(a, 0, "sqrt")))}; });
  reg(M, "fmod", [](Interp&, Values& a) { return Values{Value::number(std::fmod(check_num(a, 0, "fmod"), check_num(a, 1, "fmod")))}; });
  reg(M, "tointeger", [](Interp&, Values& a) {
    Value v = arg_at(a, 0);
    int64_t i;
    if (v.t == Value::Int) return Values{v};
    if (v.t == Value::Num && float_is_int(v.n, &i)) return Values{Value::integer(i)};
    return Values{Value()};
  });
  auto minmax = [](bool mx) {
    return [mx](Interp&, Values& a) {
      if (a.empty()) throw LuaError("bad argument #1 to 'max' (number expected)");
      Value best = a[0];
      for (size_t i = 1; i < a.size(); ++i) {
        const bool gt = a[i].as_double() > best.as_double();
        if (mx ? gt : a[i].as_double() < best.as_double()) best = a[i];
      }
      return Values{best};
    };
  };
  reg(M, "max", minmax(true));
  reg(M, "min", minmax(false));
  auto rng = std::make_shared<std::mt19937_64>(0x5eed);
  reg(M, "randomseed", [rng](Interp&, Values& a) {
    rng->seed(a.empty() ? 0x5eed : (uint64_t)check_int(a, 0, "randomseed"));
    return Values{};
  });
  reg(M, "random", [rng](Interp&, Values& a) {
    if (a.empty()) return Values{Value::number(std::uniform_real_distribution<double>(0.0, 1.0)(*rng))};
    int64_t lo = 1, hi = check_int(a, 0, "random");
    if (a.size() > 1) { lo = hi; hi = check_int(a, 1, "random"); }
    if (lo > hi) throw LuaError("bad argument to 'random' (interval is empty)");
    return Values{Value::integer(std::uniform_int_distribution<int64_t>(lo, hi)(*rng))};
  });

  // os
  auto O = std::make_shared<Table>();
  G->set(Value::string("os"), Value::table(O));
  reg(O, "time", [](Interp&, Values&) { return Values{Value::integer((int64_t)time(nullptr))}; });
  reg(O, "clock", [](Interp&, Values&) { return Values{Value::number((double)clock() / CLOCKS_PER_SEC)}; });
  reg(O, "getenv", [](Interp&, Values& a) {
    const char* v = getenv(check_str(a, 0, "getenv").c_str());
    return Values{v ? Value::string(v) : Value()};
  });
  // ---- the rest of the standard library (luaL_openlibs in the reference, splinter_cli_cmd_lua.c:395)
  // table.sort / table.move
  auto lua_less = [](Interp& I, const Value& a, const Value& b) -> bool {
    if (a.t == Value::Int && b.t == Value::Int) return a.i < b.i;
    if (a.is_num() && b.is_num()) return a.as_double() < b.as_double();
    if (a.t == Value::Str && b.t == Value::Str) return *a.s < *b.s;
    Value mm = I.metamethod(a, "__lt");
    if (mm.t == Value::Nil) mm = I.metamethod(b, "__lt");
    if (mm.t == Value::Nil)
      throw LuaError(std::string("attempt to compare ") + type_name(a) + " with " + type_name(b));
    Values r = I.call(mm, {a, b});
    return !r.empty() && r[0].truthy();
  };
  reg(T, "sort", [lua_less](Interp& I, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) throw LuaError("bad argument #1 to 'sort' (table expected)");
    Value cmp = arg_at(a, 1);
    if (cmp.t != Value::Nil && cmp.t != Value::Fn) throw LuaError("bad argument #2 to 'sort' (function expected)");
    const int64_t n = t.tab->length();
    std::vector<Value> v((size_t)n), tmp((size_t)n);
    for (int64_t i = 0; i < n; ++i) v[(size_t)i] = t.tab->get(Value::integer(i + 1));
    auto less = [&](const Value& x, const Value& y) {
      if (cmp.t == Value::Fn) {
        Values r = I.call(cmp, {x, y});
        return !r.empty() && r[0].truthy();
      }
      return lua_less(I, x, y);
    };
    // bottom-up merge sort: O(n log n) comparisons, and an inconsistent order function (which Lua
    // reports or tolerates) cannot run it out of bounds the way it can std::sort
    for (size_t w = 1; w < v.size(); w *= 2) {
      for (size_t lo = 0; lo < v.size(); lo += 2 * w) {
        const size_t mid = std::min(lo + w, v.size()), hi = std::min(lo + 2 * w, v.size());
        size_t i = lo, j = mid, k = lo;
        while (i < mid && j < hi) tmp[k++] = less(v[j], v[i]) ? v[j++] : v[i++];
        while (i < mid) tmp[k++] = v[i++];
        while (j < hi) tmp[k++] = v[j++];
      }
      v.swap(tmp);
    }
    for (int64_t i = 0; i < n; ++i) t.tab->set(Value::integer(i + 1), v[(size_t)i]);
    return Values{};
  });
  reg(T, "move", [](Interp&, Values& a) {
    Value a1 = arg_at(a, 0);
    if (a1.t != Value::Tab) throw LuaError("bad argument #1 to 'move' (table expected)");
    const int64_t f = check_int(a, 1, "move"), e = check_int(a, 2, "move"), t = check_int(a, 3, "move");
    Value a2 = a.size() > 4 && a[4].t != Value::Nil ? a[4] : a1;
    if (a2.t != Value::Tab) throw LuaError("bad argument #5 to 'move' (table expected)");
    if (e >= f) {
      if (t > e || t <= f || a1.tab != a2.tab)
        for (int64_t i = 0; i <= e - f; ++i) a2.tab->set(Value::integer(t + i), a1.tab->get(Value::integer(f + i)));
      else
        for (int64_t i = e - f; i >= 0; --i) a2.tab->set(Value::integer(t + i), a1.tab->get(Value::integer(f + i)));
    }
    return Values{a2};
  });
  reg(T, "pack", [](Interp&, Values& a) {
    auto t = std::make_shared<Table>();
    for (size_t i = 0; i < a.size(); ++i) t->set(Value::integer((int64_t)i + 1), a[i]);
    t->set(Value::string("n"), Value::integer((int64_t)a.size()));
    return Values{Value::table(t)};
  });

  // math.type / math.ult
  reg(M, "type", [](Interp&, Values& a) {
    if (a.empty()) throw LuaError("bad argument #1 to 'type' (value expected)");
    const Value v = a[0];
    return Values{v.t == Value::Int ? Value::string("integer") : v.t == Value::Num ? Value::string("float") : Value()};
  });
  reg(M, "ult", [](Interp&, Values& a) {
    return Values{Value::boolean((uint64_t)check_int(a, 0, "ult") < (uint64_t)check_int(a, 1, "ult"))};
  });
  reg(M, "exp", [](Interp&, Values& a) { return Values{Value::number(std::exp(check_num(a, 0, "exp")))}; });
  reg(M, "log", [](Interp&, Values& a) {
    const double x = check_num(a, 0, "log");
    if (a.size() < 2 || a[1].t == Value::Nil) return Values{Value::number(std::log(x))};
    const double b = check_num(a, 1, "log");
    return Values{Value::number(b == 2.0 ? std::log2(x) : b == 10.0 ? std::log10(x) : std::log(x) / std::log(b))};
  });
  for (auto& [nm, fn] : std::vector<std::pair<const char*, double (*)(double)>>{
           {"sin", std::sin}, {"cos", std::cos}, {"tan", std::tan}, {"asin", std::asin}, {"acos", std::acos}})
    reg(M, nm, [fn, nm](Interp&, Values& a) { return Values{Value::number(fn(check_num(a, 0, nm)))}; });
  reg(M, "atan", [](Interp&, Values& a) {
    const double y = check_num(a, 0, "atan"), x = a.size() > 1 && a[1].t != Value::Nil ? check_num(a, 1, "atan") : 1.0;
    return Values{Value::number(std::atan2(y, x))};
  });
  reg(M, "modf", [](Interp&, Values& a) {
    double ip = 0;
    const double fp = std::modf(check_num(a, 0, "modf"), &ip);
    int64_t i;
    return Values{float_is_int(ip, &i) ? Value::number(ip) : Value::number(ip), Value::number(fp)};
  });

  // os.date / os.time(table) / os.remove / os.rename / os.exit / os.difftime / os.tmpname
  reg(O, "date", [](Interp&, Values& a) {
    std::string fmt = a.size() > 0 && a[0].t != Value::Nil ? check_str(a, 0, "date") : "%c";
    time_t t = a.size() > 1 && a[1].t != Value::Nil ? (time_t)check_int(a, 1, "date") : time(nullptr);
    bool utc = false;
    if (!fmt.empty() && fmt[0] == '!') { utc = true; fmt = fmt.substr(1); }
    struct tm tmv;
    if (!(utc ? gmtime_r(&t, &tmv) : localtime_r(&t, &tmv))) return Values{Value()};
    if (fmt.rfind("*t", 0) == 0) {
      auto r = std::make_shared<Table>();
      const std::pair<const char*, int> f[] = {{"year", tmv.tm_year + 1900}, {"month", tmv.tm_mon + 1},
                                               {"day", tmv.tm_mday}, {"hour", tmv.tm_hour}, {"min", tmv.tm_min},
                                               {"sec", tmv.tm_sec}, {"wday", tmv.tm_wday + 1},
                                               {"yday", tmv.tm_yday + 1}};
      for (auto& kv : f) r->set(Value::string(kv.first), Value::integer(kv.second));
      r->set(Value::string("isdst"), Value::boolean(tmv.tm_isdst > 0));
      return Values{Value::table(r)};
    }
    char buf[512];
    const size_t n = strftime(buf, sizeof buf, fmt.c_str(), &tmv);
    return Values{Value::string(std::string(buf, n))};
  });
  reg(O, "time", [](Interp&, Values& a) {
    Value t = arg_at(a, 0);
    if (t.t != Value::Tab) return Values{Value::integer((int64_t)time(nullptr))};
    auto field = [&](const char* k, int dflt) -> int {
      Value v = t.tab->get(Value::string(k));
      if (v.t == Value::Nil) {
        if (dflt < 0) throw LuaError(std::string("field '") + k + "' missing in date table");
        return dflt;
      }
      return (int)toint_strict(v, "time");
    };
    struct tm tmv {};
    tmv.tm_year = field("year", -1) - 1900;
    tmv.tm_mon = field("month", -1) - 1;
    tmv.tm_mday = field("day", -1);
    tmv.tm_hour = field("hour", 12);
    tmv.tm_min = field("min", 0);
    tmv.tm_sec = field("sec", 0);
    Value dst = t.tab->get(Value::string("isdst"));
    tmv.tm_isdst = dst.t == Value::Nil ? -1 : dst.truthy();
    return Values{Value::integer((int64_t)mktime(&tmv))};
  });
  reg(O, "difftime", [](Interp&, Values& a) {
    return Values{Value::number(difftime((time_t)check_int(a, 0, "difftime"),
                                         a.size() > 1 ? (time_t)check_int(a, 1, "difftime") : 0))};
  });
  auto os_result = [](int rc, const std::string& what) {
    if (rc == 0) return Values{Value::boolean(true)};
    const int e = errno;
    return Values{Value(), Value::string(what + ": " + strerror(e)), Value::integer(e)};
  };
  reg(O, "remove", [os_result](Interp&, Values& a) {
    const std::string p = check_str(a, 0, "remove");
    return os_result(::remove(p.c_str()), p);
  });
  reg(O, "rename", [os_result](Interp&, Values& a) {
    const std::string p = check_str(a, 0, "rename"), q = check_str(a, 1, "rename");
    return os_result(::rename(p.c_str(), q.c_str()), p);
  });
  reg(O, "tmpname", [](Interp&, Values&) {
    char buf[] = "/tmp/lua_XXXXXX";
    const int fd = mkstemp(buf);
    if (fd < 0) throw LuaError("unable to generate a unique filename");
    ::close(fd);
    return Values{Value::string(buf)};
  });
  reg(O, "exit", [](Interp& I, Values& a) -> Values {
    Value c = arg_at(a, 0);
    const int code = c.t == Value::Nil || (c.t == Value::Bool && c.b) ? 0
                     : c.t == Value::Bool                             ? 1
                                                                      : (int)toint_strict(c, "exit");
    I.out("");
    fflush(stdout);
    fflush(stderr);
    std::exit(code);
  });

  // io: files are tables carrying their FILE* (metatable FILE* with the methods)
  auto FM = std::make_shared<Table>();   // file metatable
  auto FMI = std::make_shared<Table>();  // its __index: the methods
  FM->set(Value::string("__index"), Value::table(FMI));
  FM->set(Value::string("__name"), Value::string("FILE*"));
  auto mkfile = [FM](FILE* fp, bool std_stream) {
    auto t = std::make_shared<Table>();
    t->set(Value::string("__fp"), Value::integer((int64_t)(intptr_t)fp));
    if (std_stream) t->set(Value::string("__std"), Value::boolean(true));
    t->meta = FM;
    return Value::table(t);
  };
  auto fp_of = [](const Value& f, const char* fn) -> FILE* {
    if (f.t != Value::Tab) throw LuaError(std::string("bad argument #1 to '") + fn + "' (FILE* expected)");
    Value p = f.tab->get(Value::string("__fp"));
    if (p.t != Value::Int) throw LuaError(std::string("bad argument #1 to '") + fn + "' (FILE* expected)");
    if (!p.i) throw LuaError("attempt to use a closed file");
    return (FILE*)(intptr_t)p.i;
  };
  // one read format on fp: l / L / n / a / count; nil at end of input
  auto read_one = [](FILE* fp, const Value& fmt) -> Value {
    if (fmt.is_num()) {
      const int64_t n = fmt.t == Value::Int ? fmt.i : (int64_t)fmt.n;
      std::string b((size_t)std::max<int64_t>(n, 0), '\0');
      const size_t got = n > 0 ? fread(&b[0], 1, (size_t)n, fp) : 0;
      if (n > 0 && got == 0) return Value();
      b.resize(got);
      return Value::string(b);
    }
    std::string f = fmt.t == Value::Str ? *fmt.s : "l";
    if (!f.empty() && f[0] == '*') f = f.substr(1);
    const char c = f.empty() ? 'l' : f[0];
    if (c == 'a') {
      std::string b;
      char buf[4096];
      size_t n;
      while ((n = fread(buf, 1, sizeof buf, fp)) > 0) b.append(buf, n);
      return Value::string(b);
    }
    if (c == 'n') {
      double d;
      if (fscanf(fp, "%lf", &d) != 1) return Value();
      int64_t i;
      return float_is_int(d, &i) && std::floor(d) == d && std::fabs(d) < 9e15 ? Value::integer(i) : Value::number(d);
    }
    if (c == 'l' || c == 'L') {
      std::string b;
      int ch;
      bool any = false;
      while ((ch = fgetc(fp)) != EOF) {
        any = true;
        if (ch == '\n') {
          if (c == 'L') b += '\n';
          break;
        }
        b += (char)ch;
      }
      return any ? Value::string(b) : Value();
    }
    throw LuaError("bad argument to 'read' (invalid format)");
  };
  auto file_read = [fp_of, read_one](Interp&, Values& a) {
    FILE* fp = fp_of(arg_at(a, 0), "read");
    Values r;
    if (a.size() <= 1) return Values{read_one(fp, Value::string("l"))};
    for (size_t i = 1; i < a.size(); ++i) {
      r.push_back(read_one(fp, a[i]));
      if (r.back().t == Value::Nil) break;
    }
    return r;
  };
  auto write_to = [](Interp& I, FILE* fp, Values& a, size_t from) {
    for (size_t i = from; i < a.size(); ++i) {
      if (a[i].t != Value::Str && !a[i].is_num())
        throw LuaError("bad argument #" + std::to_string(i + 1 - from) + " to 'write' (string expected)");
      const std::string s = tostring(a[i]);
      if (fp == stdout) I.out(s);
      else fwrite(s.data(), 1, s.size(), fp);
    }
  };
  reg(FMI, "read", file_read);
  reg(FMI, "write", [fp_of, write_to](Interp& I, Values& a) {
    write_to(I, fp_of(arg_at(a, 0), "write"), a, 1);
    return Values{arg_at(a, 0)};
  });
  reg(FMI, "close", [fp_of](Interp&, Values& a) {
    FILE* fp = fp_of(arg_at(a, 0), "close");
    if (a[0].tab->get(Value::string("__std")).truthy()) return Values{Value(), Value::string("cannot close standard file")};
    fclose(fp);
    a[0].tab->set(Value::string("__fp"), Value::integer(0));
    return Values{Value::boolean(true)};
  });
  reg(FMI, "flush", [fp_of](Interp&, Values& a) {
    fflush(fp_of(arg_at(a, 0), "flush"));
    return Values{arg_at(a, 0)};
  });
  reg(FMI, "seek", [fp_of](Interp&, Values& a) {
    FILE* fp = fp_of(arg_at(a, 0), "seek");
    const std::string wh = a.size() > 1 && a[1].t != Value::Nil ? check_str(a, 1, "seek") : "cur";
    const long off = a.size() > 2 ? (long)check_int(a, 2, "seek") : 0;
    const int w = wh == "set" ? SEEK_SET : wh == "end" ? SEEK_END : SEEK_CUR;
    if (fseek(fp, off, w) != 0) return Values{Value(), Value::string(strerror(errno))};
    return Values{Value::integer((int64_t)ftell(fp))};
  });
  auto lines_iter = [read_one](FILE* fp, bool close_at_end, Value fmt) {
    auto st = std::make_shared<FILE*>(fp);
    return make_native("lines_iterator", [st, close_at_end, fmt, read_one](Interp&, Values&) {
      if (!*st) return Values{Value()};
      Value v = read_one(*st, fmt);
      if (v.t == Value::Nil && close_at_end) {
        fclose(*st);
        *st = nullptr;
      }
      return Values{v};
    });
  };
  reg(FMI, "lines", [fp_of, lines_iter](Interp&, Values& a) {
    return Values{lines_iter(fp_of(arg_at(a, 0), "lines"), false, a.size() > 1 ? a[1] : Value::string("l"))};
  });
  FM->set(Value::string("__tostring"), make_native("tostring", [](Interp&, Values& a) {
    Value p = arg_at(a, 0).t == Value::Tab ? a[0].tab->get(Value::string("__fp")) : Value();
    char b[64];
    if (p.t == Value::Int && p.i) snprintf(b, sizeof b, "file (%p)", (void*)(intptr_t)p.i);
    else snprintf(b, sizeof b, "file (closed)");
    return Values{Value::string(b)};
  }));
  auto IO = std::make_shared<Table>();
  G->set(Value::string("io"), Value::table(IO));
  Value io_stdout = mkfile(stdout, true), io_stdin = mkfile(stdin, true), io_stderr = mkfile(stderr, true);
  IO->set(Value::string("stdout"), io_stdout);
  IO->set(Value::string("stdin"), io_stdin);
  IO->set(Value::string("stderr"), io_stderr);
  reg(IO, "write", [write_to, io_stdout](Interp& I, Values& a) {
    write_to(I, stdout, a, 0);
    return Values{io_stdout};
  });
  reg(IO, "read", [file_read, io_stdin](Interp& I, Values& a) {
    Values b{io_stdin};
    b.insert(b.end(), a.begin(), a.end());
    return file_read(I, b);
  });
  reg(IO, "open", [mkfile](Interp&, Values& a) {
    const std::string path = check_str(a, 0, "open");
    const std::string mode = a.size() > 1 && a[1].t != Value::Nil ? check_str(a, 1, "open") : "r";
    if (mode.empty() || !strchr("rwa", mode[0])) throw LuaError("bad argument #2 to 'open' (invalid mode)");
    FILE* fp = fopen(path.c_str(), mode.c_str());
    if (!fp) {
      const int e = errno;
      return Values{Value(), Value::string(path + ": " + strerror(e)), Value::integer(e)};
    }
    return Values{mkfile(fp, false)};
  });
  reg(IO, "close", [fp_of](Interp&, Values& a) {
    FILE* fp = fp_of(arg_at(a, 0), "close");
    fclose(fp);
    a[0].tab->set(Value::string("__fp"), Value::integer(0));
    return Values{Value::boolean(true)};
  });
  reg(IO, "lines", [lines_iter](Interp&, Values& a) {
    if (a.empty() || a[0].t == Value::Nil) return Values{lines_iter(stdin, false, Value::string("l"))};
    const std::string path = check_str(a, 0, "lines");
    FILE* fp = fopen(path.c_str(), "r");
    if (!fp) throw LuaError(path + ": " + strerror(errno));
    return Values{lines_iter(fp, true, a.size() > 1 ? a[1] : Value::string("l"))};
  });
  reg(IO, "type", [](Interp&, Values& a) {
    Value f = arg_at(a, 0);
    if (f.t != Value::Tab) return Values{Value()};
    Value p = f.tab->get(Value::string("__fp"));
    if (p.t != Value::Int) return Values{Value()};
    return Values{Value::string(p.i ? "file" : "closed file")};
  });

  // load / loadstring / dofile: compile a chunk into a vararg function of the global scope
  auto compile = [](Interp& I, const std::string& src, const std::string& name, const Value* env = nullptr) -> Value {
    if (src.find("_ENV") != std::string::npos) I.env_used = true;
    Parser P(src, name);
    auto body = std::make_shared<FuncBody>();
    body->block = P.block();
    if (P.cur.t != T_EOF) P.err("'<eof>' expected");
    body->vararg = true;
    body->name = name;
    auto f = std::make_shared<Function>();
    f->body = body;
    f->env = I.root;
    if (env) {  // load(chunk, name, mode, env): the chunk's free names resolve in `env` (its _ENV upvalue)
      I.env_used = true;
      auto sc = std::make_shared<Scope>();
      sc->parent = I.root;
      sc->vars["_ENV"] = std::make_shared<Value>(*env);
      f->env = sc;
    }
    f->name = name;
    return Value::function(f);
  };
  auto load_fn = [compile](Interp& I, Values& a) {
    Value c = arg_at(a, 0);
    std::string src;
    if (c.t == Value::Str) {
      src = *c.s;
    } else if (c.t == Value::Fn) {
      for (;;) {
        Values piece = I.call(c, {});
        if (piece.empty() || piece[0].t == Value::Nil || (piece[0].t == Value::Str && piece[0].s->empty())) break;
        if (piece[0].t != Value::Str) return Values{Value(), Value::string("reader function must return a string")};
        src += *piece[0].s;
      }
    } else {
      throw LuaError("bad argument #1 to 'load' (string expected)");
    }
    const std::string name = a.size() > 1 && a[1].t == Value::Str ? *a[1].s : "=(load)";
    if (a.size() > 2 && a[2].t == Value::Str && a[2].s->find('t') == std::string::npos)
      return Values{Value(), Value::string("attempt to load a text chunk (mode is '" + *a[2].s + "')")};
    try {
      return Values{compile(I, src, name, a.size() > 3 ? &a[3] : nullptr)};
    } catch (const LuaError& e) {
      return Values{Value(), Value::string(e.what())};
    }
  };
  reg(G, "load", load_fn);
  reg(G, "loadstring", load_fn);
  auto slurp = [](const std::string& path) {
    FILE* fp = fopen(path.c_str(), "rb");
    if (!fp) throw LuaError("cannot open " + path);
    std::string src;
    char buf[4096];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, fp)) > 0) src.append(buf, n);
    fclose(fp);
    if (src.rfind("#", 0) == 0) src = "--" + src;  // shebang line
    return src;
  };
  reg(G, "loadfile", [compile, slurp](Interp& I, Values& a) {
    const std::string path = check_str(a, 0, "loadfile");
    try {
      return Values{compile(I, slurp(path), path, a.size() > 2 ? &a[2] : nullptr)};
    } catch (const LuaError& e) {
      return Values{Value(), Value::string(e.what())};
    }
  });
  reg(G, "dofile", [compile, slurp](Interp& I, Values& a) {
    const std::string path = check_str(a, 0, "dofile");
    return I.call(compile(I, slurp(path), path), {});
  });

  // utf8
  auto U = std::make_shared<Table>();
  G->set(Value::string("utf8"), Value::table(U));
  U->set(Value::string("charpattern"), Value::string(std::string("[\x00-\x7F\xC2-\xFD][\x80-\xBF]*", 14)));
  auto enc = [](int64_t cp) {
    if (cp < 0 || cp > 0x7FFFFFFF) throw LuaError("bad argument to 'char' (value out of range)");
    std::string o;
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    return o;
  };
  // decode one code point at byte i (0-based); returns its length, 0 if invalid
  auto dec = [](const std::string& s, size_t i, int64_t* cp) -> size_t {
    const unsigned char c = (unsigned char)s[i];
    size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (!n || i + n > s.size()) return 0;
    int64_t v = n == 1 ? c : n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
    for (size_t k = 1; k < n; ++k) {
      const unsigned char d = (unsigned char)s[i + k];
      if ((d & 0xC0) != 0x80) return 0;
      v = (v << 6) | (d & 0x3F);
    }
    static const int64_t minv[5] = {0, 0, 0x80, 0x800, 0x10000};
    if (v < minv[n] || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return 0;
    *cp = v;
    return n;
  };
  reg(U, "char", [enc](Interp&, Values& a) {
    std::string o;
    for (size_t i = 0; i < a.size(); ++i) o += enc(check_int(a, i, "char"));
    return Values{Value::string(o)};
  });
  auto posrel = [](int64_t p, size_t len) -> int64_t { return p >= 0 ? p : (int64_t)len + p + 1; };
  reg(U, "codepoint", [dec, posrel](Interp&, Values& a) {
    const std::string s = check_str(a, 0, "codepoint");
    const int64_t i = posrel(a.size() > 1 && a[1].t != Value::Nil ? check_int(a, 1, "codepoint") : 1, s.size());
    const int64_t j = posrel(a.size() > 2 && a[2].t != Value::Nil ? check_int(a, 2, "codepoint") : i, s.size());
    if (i < 1 || j > (int64_t)s.size()) {
      if (i > j) return Values{};
      throw LuaError("bad argument to 'codepoint' (out of bounds)");
    }
    Values r;
    for (size_t p = (size_t)i - 1; p < (size_t)j;) {
      int64_t cp;
      const size_t n = dec(s, p, &cp);
      if (!n) throw LuaError("invalid UTF-8 code");
      r.push_back(Value::integer(cp));
      p += n;
    }
    return r;
  });
  reg(U, "len", [dec, posrel](Interp&, Values& a) {
    const std::string s = check_str(a, 0, "len");
    int64_t i = posrel(a.size() > 1 && a[1].t != Value::Nil ? check_int(a, 1, "len") : 1, s.size());
    const int64_t j = posrel(a.size() > 2 && a[2].t != Value::Nil ? check_int(a, 2, "len") : -1, s.size());
    int64_t n = 0;
    for (size_t p = (size_t)std::max<int64_t>(i, 1) - 1; (int64_t)p < j;) {
      int64_t cp;
      const size_t k = dec(s, p, &cp);
      if (!k) return Values{Value(), Value::integer((int64_t)p + 1)};
      p += k;
      ++n;
    }
    return Values{Value::integer(n)};
  });
  reg(U, "offset", [posrel](Interp&, Values& a) {
    const std::string s = check_str(a, 0, "offset");
    const int64_t n = check_int(a, 1, "offset");
    int64_t i = a.size() > 2 && a[2].t != Value::Nil ? posrel(check_int(a, 2, "offset"), s.size())
                                                     : (n >= 0 ? 1 : (int64_t)s.size() + 1);
    auto cont = [&](int64_t p) { return p >= 1 && p <= (int64_t)s.size() && (((unsigned char)s[p - 1]) & 0xC0) == 0x80; };
    if (n == 0) {
      while (i > 1 && cont(i)) --i;
      return Values{Value::integer(i)};
    }
    if (cont(i)) throw LuaError("initial position is a continuation byte");
    int64_t k = n;
    if (k > 0) {
      --k;
      while (k > 0 && i <= (int64_t)s.size()) {
        ++i;
        while (cont(i)) ++i;
        --k;
      }
    } else {
      while (k < 0 && i > 1) {
        --i;
        while (i > 1 && cont(i)) --i;
        ++k;
      }
    }
    if (k != 0) return Values{Value()};
    return Values{Value::integer(i)};
  });
  reg(U, "codes", [dec](Interp&, Values& a) {
    const std::string s = check_str(a, 0, "codes");
    auto it = make_native("codes_iterator", [dec](Interp&, Values& b) {
      const std::string str = *arg_at(b, 0).s;
      int64_t p = arg_at(b, 1).t == Value::Int ? b[1].i : 0;  // 1-based position of the previous code
      if (p > 0) {
        int64_t cp;
        const size_t n = dec(str, (size_t)p - 1, &cp);
        p += n ? (int64_t)n : 1;
      } else {
        p = 1;
      }
      if (p > (int64_t)str.size()) return Values{Value()};
      int64_t cp;
      if (!dec(str, (size_t)p - 1, &cp)) throw LuaError("invalid UTF-8 code");
      return Values{Value::integer(p), Value::integer(cp)};
    });
    return Values{it, Value::string(s), Value::integer(0)};
  });


  // string.pack / string.unpack / string.packsize (Lua 5.4 sec. 6.4.2): < > = endianness, ![n] maximum
  // alignment, b B h H l L j J T i[n] I[n] (n = 1..16) integers, f d n floats, s[n] length-prefixed and
  // z zero-terminated strings, x one pad byte, X<op> alignment to op, spaces ignored
  struct PackOpt {
    char k;       // 'i' signed, 'u' unsigned, 'f' float, 'd' double, 's' prefixed string, 'z', 'x' pad, 'X' align, ' ' none
    int size;     // bytes (the length prefix for 's')
    int align;    // alignment requirement (already limited by the maximum alignment)
  };
  struct PackState {
    const std::string& fmt;
    size_t p = 0;
    bool little = true;
    int maxalign = 1;
    explicit PackState(const std::string& f) : fmt(f) {}
    int num(int dflt) {
      if (p >= fmt.size() || !isdigit((unsigned char)fmt[p])) return dflt;
      int n = 0;
      while (p < fmt.size() && isdigit((unsigned char)fmt[p]) && n < 1000) n = n * 10 + (fmt[p++] - '0');
      return n;
    }
    int isize(int dflt, const char* fn) {
      const int n = num(dflt);
      if (n < 1 || n > 16) throw LuaError(std::string("bad argument #1 to '") + fn + "' (integral size (" +
                                          std::to_string(n) + ") out of limits [1,16])");
      return n;
    }
    // next option; false at the end of the format
    bool next(PackOpt* o, const char* fn) {
      for (;;) {
        if (p >= fmt.size()) return false;
        const char c = fmt[p++];
        o->align = 1;
        switch (c) {
          case ' ': continue;
          case '<': case '=': little = true; continue;
          case '>': little = false; continue;
          case '!': maxalign = num(8); continue;
          case 'b': *o = {'i', 1, 1}; break;
          case 'B': *o = {'u', 1, 1}; break;
          case 'h': *o = {'i', 2, 2}; break;
          case 'H': *o = {'u', 2, 2}; break;
          case 'l': case 'j': *o = {'i', 8, 8}; break;
          case 'L': case 'J': case 'T': *o = {'u', 8, 8}; break;
          case 'i': { const int n = isize(4, fn); *o = {'i', n, n}; break; }
          case 'I': { const int n = isize(4, fn); *o = {'u', n, n}; break; }
          case 'f': *o = {'f', 4, 4}; break;
          case 'd': case 'n': *o = {'d', 8, 8}; break;
          case 's': { const int n = isize(8, fn); *o = {'s', n, n}; break; }
          case 'z': *o = {'z', 0, 1}; return true;
          case 'x': *o = {'x', 1, 1}; return true;
          case 'X': {
            PackOpt t{};
            const size_t at = p;
            if (!next(&t, fn) || t.k == 'z' || t.k == 's' || t.k == 'x' || t.k == 'X' || t.size == 0) {
              p = at;
              throw LuaError(std::string("bad argument #1 to '") + fn + "' (invalid next option for option 'X')");
            }
            *o = {'X', 0, t.size};
            break;
          }
          default:
            throw LuaError(std::string("bad argument #1 to '") + fn + "' (invalid format option '" + c + "')");
        }
        const int al = o->align < maxalign ? o->align : maxalign;
        if (al > 1 && (al & (al - 1)))
          throw LuaError(std::string("bad argument #1 to '") + fn + "' (format asks for alignment not power of 2)");
        o->align = al;
        return true;
      }
    }
  };
  auto pad_to = [](size_t pos, int align) -> size_t { return align > 1 ? (align - pos % (size_t)align) % (size_t)align : 0; };
  auto put_int = [](std::string& out, uint64_t v, int size, bool little, bool neg) {
    std::string b((size_t)size, '\0');
    for (int i = 0; i < size; ++i) b[(size_t)i] = (char)(i < 8 ? (v >> (8 * i)) & 0xff : (neg ? 0xff : 0));
    if (!little) std::reverse(b.begin(), b.end());
    out += b;
  };
  reg(S, "pack", [pad_to, put_int](Interp&, Values& a) {
    const std::string fmt = check_str(a, 0, "pack");
    PackState st(fmt);
    std::string out;
    size_t arg = 1;
    PackOpt o{};
    while (st.next(&o, "pack")) {
      out.append(pad_to(out.size(), o.align), '\0');
      switch (o.k) {
        case 'i': case 'u': {
          const int64_t v = check_int(a, arg, "pack");
          if (o.size < 8) {
            if (o.k == 'i') {
              const int64_t lim = (int64_t)1 << (o.size * 8 - 1);
              if (v < -lim || v >= lim) throw LuaError("bad argument #" + std::to_string(arg + 1) + " to 'pack' (integer overflow)");
            } else if ((uint64_t)v >= ((uint64_t)1 << (o.size * 8))) {
              throw LuaError("bad argument #" + std::to_string(arg + 1) + " to 'pack' (unsigned overflow)");
            }
          }
          put_int(out, (uint64_t)v, o.size, st.little, o.k == 'i' && v < 0);
          ++arg;
          break;
        }
        case 'f': case 'd': {
          const double d = check_num(a, arg++, "pack");
          uint64_t bits = 0;
          if (o.k == 'f') {
            const float f = (float)d;
            uint32_t b32;
            std::memcpy(&b32, &f, 4);
            bits = b32;
          } else {
            std::memcpy(&bits, &d, 8);
          }
          put_int(out, bits, o.size, st.little, false);
          break;
        }
        case 's': {
          const std::string v = check_str(a, arg++, "pack");
          if (o.size < 8 && (uint64_t)v.size() >= ((uint64_t)1 << (o.size * 8)))
            throw LuaError("bad argument #" + std::to_string(arg) + " to 'pack' (string length does not fit in given size)");
          put_int(out, (uint64_t)v.size(), o.size, st.little, false);
          out += v;
          break;
        }
        case 'z': {
          const std::string v = check_str(a, arg++, "pack");
          if (v.find('\0') != std::string::npos)
            throw LuaError("bad argument #" + std::to_string(arg) + " to 'pack' (string contains zeros)");
          out += v;
          out += '\0';
          break;
        }
        case 'x': out += '\0'; break;
        case 'X': break;
      }
    }
    return Values{Value::string(out)};
  });
  reg(S, "packsize", [pad_to](Interp&, Values& a) {
    const std::string fmt = check_str(a, 0, "packsize");
    PackState st(fmt);
    size_t n = 0;
    PackOpt o{};
    while (st.next(&o, "packsize")) {
      if (o.k == 's' || o.k == 'z') throw LuaError("bad argument #1 to 'packsize' (variable-length format)");
      n += pad_to(n, o.align) + (size_t)o.size;
    }
    return Values{Value::integer((int64_t)n)};
  });
  reg(S, "unpack", [pad_to](Interp&, Values& a) {
    const std::string fmt = check_str(a, 0, "unpack");
    const std::string data = check_str(a, 1, "unpack");
    int64_t init = a.size() > 2 && a[2].t != Value::Nil ? check_int(a, 2, "unpack") : 1;
    if (init < 0) init = (int64_t)data.size() + init + 1;
    if (init < 1 || init - 1 > (int64_t)data.size()) throw LuaError("bad argument #3 to 'unpack' (initial position out of string)");
    size_t pos = (size_t)init - 1;
    PackState st(fmt);
    Values out;
    PackOpt o{};
    auto need = [&](size_t n) {
      if (pos + n > data.size()) throw LuaError("bad argument #2 to 'unpack' (data string too short)");
    };
    auto get_int = [&](int size, bool sign) -> uint64_t {
      need((size_t)size);
      uint64_t v = 0;
      for (int i = 0; i < size; ++i) {
        const uint8_t byte = (uint8_t)data[pos + (size_t)(st.little ? i : size - 1 - i)];
        if (i < 8) v |= (uint64_t)byte << (8 * i);
        else if (byte != ((sign && (int64_t)v < 0) ? 0xff : 0))
          throw LuaError(std::to_string(size) + "-byte integer does not fit into Lua Integer");
      }
      if (sign && size < 8 && (v >> (size * 8 - 1)) & 1) v |= ~(uint64_t)0 << (size * 8);
      pos += (size_t)size;
      return v;
    };
    while (st.next(&o, "unpack")) {
      const size_t pad = pad_to(pos, o.align);
      need(pad);
      pos += pad;
      switch (o.k) {
        case 'i': out.push_back(Value::integer((int64_t)get_int(o.size, true))); break;
        case 'u': out.push_back(Value::integer((int64_t)get_int(o.size, false))); break;
        case 'f': {
          const uint32_t b = (uint32_t)get_int(4, false);
          float f;
          std::memcpy(&f, &b, 4);
          out.push_back(Value::number(f));
          break;
        }
        case 'd': {
          const uint64_t b = get_int(8, false);
          double d;
          std::memcpy(&d, &b, 8);
          out.push_back(Value::number(d));
          break;
        }
        case 's': {
          const uint64_t n = get_int(o.size, false);
          need((size_t)n);
          out.push_back(Value::string(data.substr(pos, (size_t)n)));
          pos += (size_t)n;
          break;
        }
        case 'z': {
          const size_t e = data.find('\0', pos);
          if (e == std::string::npos) throw LuaError("bad argument #2 to 'unpack' (unfinished string for format 'z')");
          out.push_back(Value::string(data.substr(pos, e - pos)));
          pos = e + 1;
          break;
        }
        case 'x': need(1); ++pos; break;
        case 'X': break;
      }
    }
    out.push_back(Value::integer((int64_t)pos + 1));
    return out;
  });

  // debug (the subset a tree-walking interpreter can give): traceback, getinfo, get/setmetatable
  // without __metatable protection, getregistry, sethook/gethook (no hooks run), getlocal /
  // getupvalue (no indexed locals or upvalues here: nil)
  auto D = std::make_shared<Table>();
  G->set(Value::string("debug"), Value::table(D));
  registry = std::make_shared<Table>();
  reg(D, "traceback", [](Interp& I, Values& a) {
    size_t at = a.size() > 0 && a[0].t == Value::Co ? 1 : 0;  // optional thread argument
    Value m = arg_at(a, at);
    if (m.t != Value::Nil && m.t != Value::Str && !m.is_num()) return Values{m};
    std::string s = m.t == Value::Nil ? "" : (m.t == Value::Str ? *m.s : tostring(m)) + "\n";
    s += "stack traceback:\n\t" + I.chunk + ":" + std::to_string(I.line) + ": in function <" + I.chunk + ">\n\t[C]: in ?";
    return Values{Value::string(s)};
  });
  reg(D, "getinfo", [](Interp& I, Values& a) {
    size_t at = a.size() > 0 && a[0].t == Value::Co ? 1 : 0;
    Value f = arg_at(a, at);
    auto t = std::make_shared<Table>();
    t->set(Value::string("source"), Value::string("@" + I.chunk));
    t->set(Value::string("short_src"), Value::string(I.chunk));
    if (f.t == Value::Fn) {
      const bool native = (bool)f.fn->native;
      t->set(Value::string("what"), Value::string(native ? "C" : "Lua"));
      t->set(Value::string("func"), f);
      t->set(Value::string("currentline"), Value::integer(-1));
      t->set(Value::string("linedefined"), Value::integer(native ? -1 : 0));
      t->set(Value::string("nparams"), Value::integer(native ? 0 : (int64_t)f.fn->body->params.size()));
      t->set(Value::string("isvararg"), Value::boolean(native || f.fn->body->vararg));
      if (native) t->set(Value::string("source"), Value::string("=[C]")), t->set(Value::string("short_src"), Value::string("[C]"));
      if (!f.fn->name.empty()) t->set(Value::string("name"), Value::string(f.fn->name));
    } else if (f.is_num()) {
      const int64_t level = toint_strict(f, "getinfo");
      if (level < 0 || level > I.depth) return Values{Value()};
      t->set(Value::string("what"), Value::string(level == 0 ? "C" : "Lua"));
      t->set(Value::string("currentline"), Value::integer(level == 0 ? -1 : I.line));
    } else {
      throw LuaError("bad argument #1 to 'getinfo' (function or level expected)");
    }
    t->set(Value::string("nups"), Value::integer(0));
    t->set(Value::string("istailcall"), Value::boolean(false));
    return Values{Value::table(t)};
  });
  reg(D, "getmetatable", [](Interp& I, Values& a) {
    Value v = arg_at(a, 0);
    std::shared_ptr<Table> m = v.t == Value::Tab ? v.tab->meta : v.t == Value::Str ? I.string_meta : nullptr;
    return Values{m ? Value::table(m) : Value()};
  });
  reg(D, "setmetatable", [](Interp& I, Values& a) {
    Value v = arg_at(a, 0), m = arg_at(a, 1);
    if (m.t != Value::Nil && m.t != Value::Tab) throw LuaError("bad argument #2 to 'setmetatable' (nil or table expected)");
    if (v.t == Value::Tab) v.tab->meta = m.t == Value::Tab ? m.tab : nullptr;
    else if (v.t == Value::Str) I.string_meta = m.t == Value::Tab ? m.tab : nullptr;
    else throw LuaError("debug.setmetatable: only tables and strings carry metatables here");
    return Values{v};
  });
  reg(D, "getregistry", [](Interp& I, Values&) { return Values{Value::table(I.registry)}; });
  reg(D, "sethook", [](Interp&, Values&) { return Values{}; });
  reg(D, "gethook", [](Interp&, Values&) { return Values{Value()}; });
  reg(D, "getlocal", [](Interp&, Values&) { return Values{Value()}; });
  reg(D, "getupvalue", [](Interp&, Values&) { return Values{Value()}; });
  reg(D, "setupvalue", [](Interp&, Values&) { return Values{Value()}; });
  reg(D, "upvalueid", [](Interp&, Values&) { return Values{Value()}; });

  for (const char* lib : {"string", "table", "math", "os", "coroutine", "io", "utf8", "debug"})
    modules[lib] = G->get(Value::string(lib));
}

// __gc (collectgarbage): a mark phase from the roots -- globals, registry, string metatable, loaded
// modules and the scope stacks of every running or suspended call -- through tables, metatables,
// closures' scopes and coroutines; marked tables it did not reach are finalized (reverse marking
// order), as are, at close (all), the rest.  Values held only by a native function's C++ frame
// while it runs are not roots (a finalizer may then run early; the object itself stays valid).
// Errors in finalizers are dropped (warnings off).
void Interp::run_finalizers(bool all) {
  for (int round = 0; round < 64 && !finalizers.empty(); ++round) {
    std::unordered_set<const void*> seen;
    if (!all) {
      std::vector<const Table*> tw;
      std::vector<const Scope*> sw;
      std::function<void(const Value&)> val = [&](const Value& v) {
        switch (v.t) {
          case Value::Tab:
            if (v.tab && seen.insert(v.tab.get()).second) tw.push_back(v.tab.get());
            break;
          case Value::Fn:
            if (v.fn && seen.insert(v.fn.get()).second && v.fn->env && seen.insert(v.fn->env.get()).second)
              sw.push_back(v.fn->env.get());
            break;
          case Value::Co:
            if (v.co && seen.insert(v.co.get()).second) {
              val(v.co->fn);
              for (const Value& x : v.co->transfer) val(x);
            }
            break;
          default: break;
        }
      };
      auto scope = [&](const std::shared_ptr<Scope>& sc) {
        if (sc && seen.insert(sc.get()).second) sw.push_back(sc.get());
      };
      val(Value::table(globals));
      if (registry) val(Value::table(registry));
      if (string_meta) val(Value::table(string_meta));
      for (auto& m : modules) val(m.second);
      scope(root);
      for (auto* st : scope_stacks)
        for (auto& sc : *st) scope(sc);
      while (!tw.empty() || !sw.empty()) {
        if (!tw.empty()) {
          const Table* t = tw.back();
          tw.pop_back();
          for (auto& e : t->entries) {
            val(e.first);
            val(e.second);
          }
          if (t->meta) val(Value::table(t->meta));
        } else {
          const Scope* sc = sw.back();
          sw.pop_back();
          for (auto& c : sc->vars)
            if (c.second) val(*c.second);
          for (auto& x : sc->varargs) val(x);
          for (auto& x : sc->tbc) val(x);
          if (sc->parent && seen.insert(sc->parent.get()).second) sw.push_back(sc->parent.get());
        }
      }
    }
    std::vector<std::shared_ptr<Table>> dead;
    for (size_t i = finalizers.size(); i-- > 0;)
      if (all || !seen.count(finalizers[i].get())) {
        dead.push_back(std::move(finalizers[i]));
        finalizers.erase(finalizers.begin() + (long)i);
      }
    if (dead.empty()) break;
    for (auto& t : dead) {
      Value h = t->meta ? t->meta->get(Value::string("__gc")) : Value();
      if (h.t == Value::Nil) continue;
      try {
        call(h, {Value::table(t)});
      } catch (const LuaError&) {
      }
    }
    if (!all) break;  // objects a finalizer released wait for the next cycle, as in Lua
  }
}

Interp::~Interp() {
  try {
    run_finalizers(true);
  } catch (...) {
  }
  // Move every live table's and scope's contents into one graveyard first (moves destroy
  // nothing, so no registered object disappears while the sets are walked), then drop it.
  std::vector<Value> grave;
  std::vector<std::shared_ptr<Value>> cells;
  std::vector<std::shared_ptr<Scope>> parents;
  globals.reset();
  root.reset();
  modules.clear();
  string_meta.reset();
  for (Table* t : heap->tables) {
    for (auto& e : t->entries) {
      grave.push_back(std::move(e.first));
      grave.push_back(std::move(e.second));
    }
    t->entries.clear();
    t->index.clear();  // keys are copies of entries' keys: strings and tables both already moved
    if (t->meta) grave.push_back(Value::table(std::move(t->meta)));
  }
  for (Scope* s : heap->scopes) {
    for (auto& v : s->vars) cells.push_back(std::move(v.second));
    s->vars.clear();
    parents.push_back(std::move(s->parent));
    for (auto& v : s->varargs) grave.push_back(std::move(v));
    s->varargs.clear();
  }
  for (auto& c : cells)
    if (c) grave.push_back(std::move(*c));
  t_heap = prev_heap;  // objects destroyed below unregister from `heap`, which stays valid
  grave.clear();
  cells.clear();
  parents.clear();
  for (Table* t : heap->tables) t->heap = nullptr;  // still held outside the interpreter
  for (Scope* s : heap->scopes) s->heap = nullptr;
  delete heap;
}

void Interp::set_global(const std::string& name, Value v) { globals->set(Value::string(name), std::move(v)); }
Value Interp::global(const std::string& name) const { return globals->get(Value::string(name)); }

Values Interp::run(const std::string& src, const std::string& chunkname, const std::vector<std::string>& args) {
  chunk = chunkname;
  if (src.find("_ENV") != std::string::npos) env_used = true;
  Parser P(src, chunkname);
  auto body = std::make_shared<FuncBody>();
  body->block = P.block();
  if (P.cur.t != T_EOF) P.err("'<eof>' expected");
  body->vararg = true;
  body->name = "main chunk";
  auto argt = std::make_shared<Table>();
  argt->set(Value::integer(0), Value::string(chunkname));
  Values va;
  for (size_t i = 0; i < args.size(); ++i) {
    argt->set(Value::integer((int64_t)i + 1), Value::string(args[i]));
    va.push_back(Value::string(args[i]));
  }
  set_global("arg", Value::table(argt));
  auto f = std::make_shared<Function>();
  f->body = body;
  f->env = root;
  f->name = chunkname;
  return call(Value::function(f), va);
}

}  // namespace mlua
