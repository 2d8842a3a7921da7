// splinterctl / splinter_cli — command-line front end for libsplinter_amd.
//
// Same verbs, argument conventions and output formats as the reference CLI
// (/root/reference/splinter_cli_main.c:42-325 module table, 666-679 options,
// 382-401 mode selection; one file per verb in splinter_cli_cmd_*.c), written
// fresh in C++ on top of the reference-compatible C API.  Stores may be shm
// names, file paths, or "hbm:NAME" GPU arenas (same verbs everywhere).
//   * argv[0] splinterctl / splinterpctl -> one-shot; anything else -> REPL
//   * prefix matching of verbs ("getx" runs get), ~/.splinterrc label map,
//     SPLINTER_NS_PREFIX / --prefix namespace, SPLINTER_DEFAULT_STORE,
//     SPLINTER_HISTORY_FILE / _LEN
//   * `lua` runs on minilua (Lua 5.4 subset) and `wasm` on miniwasm (MVP
//     interpreter, binary or WAT): neither Lua 5.4 nor WasmEdge is in this
//     image, so both hosts are built in (`caps` reports them).
#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fcntl.h>
#include <functional>
#include <getopt.h>
#include <libgen.h>
#include <regex.h>
#include <string>
#include <sys/mman.h>
#include <thread>
#include <sys/syscall.h>
#include <unistd.h>
#include <vector>

#include "lineedit.hpp"
#include "minilua.hpp"
#include "miniwasm.hpp"
#include <dlfcn.h>
#include "splinter_ext.h"

#ifndef SPL_BUILD_ID
#define SPL_BUILD_ID "dev"
#endif
#define SPLINTER_VERSION "1.2.0-amd"
#define DEFAULT_BUS "splinter_debug"
#define DEFAULT_SLOTS 1024
#define DEFAULT_VAL_MAXLEN 4096

namespace {

struct Label {
  std::string name;
  uint64_t mask;
};

struct Ctx {
  std::string store;
  bool connected = false;
  std::string prefix;
  std::vector<Label> labels;
  std::vector<std::string> history;
  std::string history_file;
  int history_len = 1000;
  volatile sig_atomic_t abort = 0;
} U;

using Handler = std::function<int(int, char**)>;
struct Module {
  const char* name;
  const char* help;
  Handler run;
  std::function<void()> usage;
};
std::vector<Module>& modules() {
  static std::vector<Module> m;
  return m;
}

std::string pkey(const char* k) { return U.prefix + (k ? k : ""); }

const char* type_name(unsigned t) {
  switch (t) {
    case SPL_SLOT_TYPE_VOID: return "SPL_SLOT_TYPE_VOID";
    case SPL_SLOT_TYPE_BIGINT: return "SPL_SLOT_TYPE_BIGINT";
    case SPL_SLOT_TYPE_BIGUINT: return "SPL_SLOT_TYPE_BIGUINT";
    case SPL_SLOT_TYPE_JSON: return "SPL_SLOT_TYPE_JSON";
    case SPL_SLOT_TYPE_BINARY: return "SPL_SLOT_TYPE_BINARY";
    case SPL_SLOT_TYPE_IMGDATA: return "SPL_SLOT_TYPE_IMGDATA";
    case SPL_SLOT_TYPE_AUDIO: return "SPL_SLOT_TYPE_AUDIO";
    case SPL_SLOT_TYPE_VARTEXT: return "SPL_SLOT_TYPE_VARTEXT";
    default: return "SPL_SLOT_TYPE_UNKNOWN";
  }
}

unsigned type_from_name(const char* s) {
  struct { const char* n; unsigned v; } t[] = {
      {"void", SPL_SLOT_TYPE_VOID}, {"bigint", SPL_SLOT_TYPE_BIGINT}, {"biguint", SPL_SLOT_TYPE_BIGUINT},
      {"json", SPL_SLOT_TYPE_JSON}, {"binary", SPL_SLOT_TYPE_BINARY}, {"img", SPL_SLOT_TYPE_IMGDATA},
      {"audio", SPL_SLOT_TYPE_AUDIO}, {"vartext", SPL_SLOT_TYPE_VARTEXT}};
  for (auto& e : t)
    if (!strcasecmp(s, e.n)) return e.v;
  return 0;
}

bool parse_mask(const char* s, uint64_t* out) {
  for (auto& l : U.labels)
    if (!strcasecmp(l.name.c_str(), s)) { *out = l.mask; return true; }
  char* end = nullptr;
  errno = 0;
  uint64_t v = strtoull(s, &end, 0);
  if (errno || end == s || *end) return false;
  *out = v;
  return true;
}

std::string binary(uint64_t v) {
  if (!v) return "0";
  std::string s;
  for (int b = 63; b >= 0; --b)
    if (!s.empty() || (v >> b & 1)) s.push_back((v >> b & 1) ? '1' : '0');
  return s;
}

bool need_store(const char* mod) {
  if (!U.connected) { fprintf(stderr, "%s: not connected to a store.\n", mod); return false; }
  return true;
}

void load_rc(const std::string& path_in) {
  std::string path = path_in;
  if (path.empty()) {
    const char* home = getenv("HOME");
    if (!home) return;
    path = std::string(home) + "/.splinterrc";
  }
  FILE* f = fopen(path.c_str(), "r");
  if (!f) {
    if (!path_in.empty()) fprintf(stderr, "splinterctl: cannot open rc file '%s': %s\n", path.c_str(), strerror(errno));
    return;
  }
  char line[256];
  while (fgets(line, sizeof line, f) && U.labels.size() < 63) {
    if (line[0] == '#' || line[0] == '\n' || line[0] == '\r') continue;
    char name[64], mask[32];
    if (sscanf(line, "%63s %31s", name, mask) == 2) {
      char* end;
      errno = 0;
      uint64_t m = strtoull(mask, &end, 0);
      if (!errno && end != mask) U.labels.push_back({name, m});
    }
  }
  fclose(f);
}

// ------------------------------------------------------------ tokenizer --
std::vector<std::string> tokenize(const std::string& line) {
  std::vector<std::string> out;
  std::string cur;
  bool in = false, any = false;
  char q = 0;
  for (size_t i = 0; i < line.size(); ++i) {
    char c = line[i];
    if (q) {
      if (c == q) { q = 0; continue; }
      if (c == '\\' && q == '"' && i + 1 < line.size()) { cur.push_back(line[++i]); continue; }
      cur.push_back(c);
      continue;
    }
    if (c == '"' || c == '\'') { q = c; in = any = true; continue; }
    if (c == '\\' && i + 1 < line.size()) { cur.push_back(line[++i]); in = any = true; continue; }
    if (isspace((unsigned char)c)) {
      if (in) { out.push_back(cur); cur.clear(); in = false; }
      continue;
    }
    cur.push_back(c);
    in = any = true;
  }
  if (in || (any && !cur.empty())) out.push_back(cur);
  return out;
}

int find_module(const char* name) {
  auto& m = modules();
  for (size_t i = 0; i < m.size(); ++i)
    if (!strcmp(name, m[i].name)) return (int)i;
  for (size_t i = 0; i < m.size(); ++i)  // reference: prefix match on the module name
    if (!strncmp(name, m[i].name, strlen(m[i].name))) return (int)i;
  return -1;
}

int run_argv(std::vector<std::string> args) {
  if (args.empty()) return 0;
  int idx = find_module(args[0].c_str());
  if (idx < 0) {
    fprintf(stderr, "Unknown command: %s\n", args[0].c_str());
    return 1;
  }
  std::vector<char*> av;
  for (auto& a : args) av.push_back(&a[0]);
  av.push_back(nullptr);
  optind = 0;  // glibc: full re-initialisation, so options after operands are permuted again
  opterr = 1;
  return modules()[(size_t)idx].run((int)args.size(), av.data());
}

// --------------------------------------------------------------- verbs --
int cmd_clear(int, char**) {
  printf("\033[H\033[2J");
  fflush(stdout);
  return 0;
}

int cmd_config(int argc, char** argv) {
  if (!need_store("config")) return 1;
  if (argc == 1) {
    splinter_header_snapshot_t s{};
    splinter_get_header_snapshot(&s);
    printf("magic:       %u\n", s.magic);
    printf("version:     %u\n", s.version);
    printf("slots:       %u\n", s.slots);
    printf("alignment:   %zu\n", (size_t)alignof(struct splinter_slot));
    printf("max_val_sz:  %u\n", s.max_val_sz);
    printf("epoch:       %lu\n", (unsigned long)s.epoch);
    printf("auto_scrub : %u\n", (s.core_flags & SPL_SYS_AUTO_SCRUB) ? 1 : 0);
    printf("mop:         %d\n", splinter_get_mop());
    uint32_t slots, mv, stride;
    spl_store_geometry(spl_store_current(), &slots, &mv, &stride);
    printf("backend:     %s\n", spl_store_backend(spl_store_current()));
    printf("slot_stride: %u (%s)\n", stride, stride == 3200 ? "embeddings" : "plain");
    puts("");
    return 0;
  }
  if (argc == 3 && (!strncmp(argv[1], "av", 2) || !strcmp(argv[1], "mop"))) {
    int v = atoi(argv[2]);
    if (splinter_set_mop((unsigned)v) != 0) {
      fprintf(stderr, "Invalid setting flag (0 = off, 1 = hybrid, 2 = boil)");
      return 1;
    }
    return 0;
  }
  fprintf(stderr, "Invalid configuration token: %s\n", argc > 1 ? argv[1] : "");
  return 1;
}

int cmd_get(int argc, char** argv) {
  if (argc != 2) { fprintf(stderr, "Usage: get <key_name>\n"); return 1; }
  if (!need_store("get")) return 1;
  std::string key = pkey(argv[1]);
  std::vector<char> buf(4097, 0);
  size_t n = 0;
  if (splinter_get(key.c_str(), buf.data(), 4096, &n) != 0) {
    fprintf(stderr, "get: unable to retrieve key '%s'\n", key.c_str());
    return 1;
  }
  splinter_slot_snapshot_t s{};
  splinter_get_slot_snapshot(key.c_str(), &s);
  if ((s.type_flag & SPL_SLOT_TYPE_BIGUINT) && n >= 8) {
    uint64_t v;
    memcpy(&v, buf.data(), 8);
    printf("%llu\n", (unsigned long long)v);
  } else {
    buf[n] = 0;
    printf("%s\n", buf.data());
  }
  puts("");
  return 0;
}

void show_head(const char* key) {
  splinter_slot_snapshot_t s{};
  splinter_get_slot_snapshot(key, &s);
  if (s.epoch == 0) { fprintf(stderr, "head: invalid key: %s\n", key); return; }
  printf("hash:       %lu\n", (unsigned long)s.hash);
  printf("epoch:      %lu\n", (unsigned long)s.epoch);
  printf("bloom:      %lu (0b%s)\n", (unsigned long)s.bloom, binary(s.bloom).c_str());
  printf("val_off:    %u\n", s.val_off);
  printf("val_len:    %u\n", s.val_len);
  printf("ctime:      %lu\n", (unsigned long)s.ctime);
  printf("atime:      %lu\n", (unsigned long)s.atime);
  printf("type:       %s\n", type_name(s.type_flag));
  printf("key:        %s\n", s.key);
  double mag = 0;
  uint32_t chk = 0;
  for (int i = 0; i < SPLINTER_EMBED_DIM; ++i) {
    mag += (double)s.embedding[i] * s.embedding[i];
    uint32_t u;
    memcpy(&u, &s.embedding[i], 4);
    chk ^= u;
  }
  printf("embed:      DIM=%d, Mag=%.4f, Checksum=0x%08x\n", SPLINTER_EMBED_DIM, std::sqrt(mag), chk);
  printf("vec[0..2]:  [%.3f, %.3f, %.3f, ...]\n", s.embedding[0], s.embedding[1], s.embedding[2]);
  puts("");
}

int cmd_head(int argc, char** argv) {
  if (argc != 2) { fprintf(stderr, "Usage: head <key_name>\n"); return 1; }
  if (!need_store("head")) return 1;
  show_head(pkey(argv[1]).c_str());
  return 0;
}

int cmd_help(int argc, char** argv) {
  const char* target = argc >= 2 ? argv[argc - 1] : nullptr;
  if (target && strcmp(target, "ext")) {
    int i = find_module(target);
    if (i < 0) { fprintf(stderr, "help: unknown module '%s'\n", target); return 1; }
    auto& m = modules()[(size_t)i];
    printf("%s: %s\n", m.name, m.help);
    if (m.usage) m.usage();
    return 0;
  }
  printf("Available commands:\n");
  for (auto& m : modules()) printf("  %-10s %s\n", m.name, m.help);
  puts("\nUse 'help <command>' for details.");
  return 0;
}

int cmd_hist(int argc, char** argv) {
  if (argc == 2 && !strcmp(argv[1], "clear")) { U.history.clear(); return 0; }
  regex_t re;
  bool filt = argc == 2 && regcomp(&re, argv[1], REG_EXTENDED | REG_NOSUB) == 0;
  for (size_t i = 0; i < U.history.size(); ++i)
    if (!filt || regexec(&re, U.history[i].c_str(), 0, nullptr, 0) == 0) printf("%4zu  %s\n", i + 1, U.history[i].c_str());
  if (filt) regfree(&re);
  return 0;
}

int cmd_list(int argc, char** argv) {
  if (!need_store("list")) return 1;
  splinter_header_snapshot_t h{};
  splinter_get_header_snapshot(&h);
  std::vector<char*> names(h.slots ? h.slots : 1);
  size_t n = 0;
  splinter_list(names.data(), names.size(), &n);
  regex_t re;
  bool filt = argc >= 2 && regcomp(&re, argv[1], REG_EXTENDED | REG_NOSUB) == 0;
  size_t max_lines = argc >= 3 ? (size_t)atol(argv[2]) : 0;
  std::vector<splinter_slot_snapshot_t> snaps;
  for (size_t i = 0; i < n; ++i) {
    std::string k(names[i]);
    if (k.empty()) continue;
    if (filt && regexec(&re, k.c_str(), 0, nullptr, 0) != 0) continue;
    splinter_slot_snapshot_t s{};
    if (splinter_get_slot_snapshot(k.c_str(), &s) == 0) snaps.push_back(s);
  }
  if (filt) regfree(&re);
  std::sort(snaps.begin(), snaps.end(), [](const auto& a, const auto& b) { return a.epoch > b.epoch; });
  printf("%-44s %-6s %-6s %s\n", "Name", "Epoch", "Len", "Type");
  for (size_t i = 0; i < snaps.size() && (!max_lines || i < max_lines); ++i)
    printf("%-44s %-6lu %-6u %s\n", snaps[i].key, (unsigned long)snaps[i].epoch, snaps[i].val_len,
           type_name(snaps[i].type_flag));
  puts("");
  return 0;
}

int cmd_set(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "Usage: set <key> <value>\n"); return 1; }
  if (!need_store("set")) return 1;
  std::string key = pkey(argv[1]);
  int rc = splinter_set(key.c_str(), argv[2], strnlen(argv[2], 4096));
  if (rc != 0) fprintf(stderr, "set: failed to set '%s': %s\n", key.c_str(), strerror(errno));
  return rc ? 1 : 0;
}

int cmd_unset(int argc, char** argv) {
  bool rec = false;
  const char* k = nullptr;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "-r")) rec = true;
    else k = argv[i];
  }
  if (!k) { fprintf(stderr, "Usage: unset [-r] <key_name>\n"); return 1; }
  if (!need_store("unset")) return 1;
  std::string key = pkey(k);
  long total = 0;
  int r = splinter_unset(key.c_str());
  if (r > 0) total += r;
  if (rec) {
    for (unsigned i = 1; i < 256; ++i) {
      std::string t = key + SPL_ORDER_ACCESSOR + std::to_string(i);
      int x = splinter_unset(t.c_str());
      if (x < 0) break;
      total += x;
    }
  }
  printf("%ld bytes deleted.\n", total);
  return r < 0 ? 1 : 0;
}

int open_store(const std::string& name) {
  if (splinter_open(name.c_str()) != 0) return -1;
  U.store = name;
  U.connected = true;
  return 0;
}

int cmd_use(int argc, char** argv) {
  if (argc != 2) { fprintf(stderr, "Usage: use <store_name>\n"); return 1; }
  splinter_close();
  U.connected = false;
  if (open_store(argv[1]) != 0) {
    fprintf(stderr, "use: unable to open '%s': %s\n", argv[1], strerror(errno));
    return 1;
  }
  return 0;
}

int cmd_watch(int argc, char** argv) {
  static option lo[] = {{"oneshot", no_argument, nullptr, 'o'}, {"group", required_argument, nullptr, 'g'},
                        {"help", no_argument, nullptr, 'h'}, {nullptr, 0, nullptr, 0}};
  bool oneshot = false;
  int group = -1, opt;
  while ((opt = getopt_long(argc, argv, "og:h", lo, nullptr)) != -1) {
    if (opt == 'o') oneshot = true;
    else if (opt == 'g') {
      group = atoi(optarg);
      if (group < 0 || group >= SPLINTER_MAX_GROUPS) {
        fprintf(stderr, "watch: invalid group. Must be 0-%d\n", SPLINTER_MAX_GROUPS - 1);
        return 1;
      }
    } else return 1;
  }
  if (!need_store("watch")) return 1;
  U.abort = 0;
  if (group >= 0) {
    uint64_t last = splinter_get_signal_count((uint8_t)group);
    while (!U.abort) {
      uint64_t cur = splinter_get_signal_count((uint8_t)group);
      if (cur != last) {
        fprintf(stdout, "Signal group %d pulsed! (Total pulses: %lu)\n", group, (unsigned long)cur);
        fflush(stdout);
        last = cur;
        if (oneshot) break;
      }
      usleep(50000);
    }
    return 0;
  }
  if (optind >= argc) {
    fprintf(stderr, "Usage: watch <key> [--oneshot] OR watch --group <id> [--oneshot]\n");
    return 1;
  }
  std::string key = pkey(argv[optind]);
  if (!oneshot) puts("Press `<ctrl> + ]` (or SIGUSR1) to leave the continuous watch loop ...");
  while (!U.abort) {
    int rc = splinter_poll(key.c_str(), 100);
    if (rc == 0) {
      std::vector<char> buf(65536, 0);
      size_t n = 0;
      if (splinter_get(key.c_str(), buf.data(), buf.size() - 1, &n) == 0) {
        fprintf(stdout, "%lu:%.*s\n", (unsigned long)n, (int)n, buf.data());
        fflush(stdout);
      }
      if (oneshot) break;
    } else if (rc == -1 && errno != ETIMEDOUT && errno != EAGAIN) {
      fprintf(stderr, "watch: invalid key: '%s'\n", key.c_str());
      return 1;
    }
  }
  return 0;
}

int cmd_init(int argc, char** argv) {
  static option lo[] = {{"slots", required_argument, nullptr, 's'}, {"length", required_argument, nullptr, 'l'},
                        {"no-embeddings", no_argument, nullptr, 'N'}, {"embeddings", no_argument, nullptr, 'E'},
                        {"help", no_argument, nullptr, 'h'}, {nullptr, 0, nullptr, 0}};
  unsigned long slots = DEFAULT_SLOTS, len = DEFAULT_VAL_MAXLEN;
  int emb = -1, opt;
  while ((opt = getopt_long(argc, argv, "s:l:NEh", lo, nullptr)) != -1) {
    if (opt == 's') slots = strtoul(optarg, nullptr, 0);
    else if (opt == 'l') len = strtoul(optarg, nullptr, 0);
    else if (opt == 'N') emb = 0;
    else if (opt == 'E') emb = 1;
    else return 1;
  }
  std::string store = optind < argc ? argv[argc - 1] : DEFAULT_BUS;
  std::string save = U.connected ? U.store : "";
  unsigned flags = emb < 0 ? 0 : (emb ? SPL_CREATE_EMBEDDINGS : SPL_CREATE_NO_EMBEDDINGS);
  const size_t stride = (emb == 0 || (emb < 0 && getenv("SPLINTER_EMBEDDINGS") &&
                                      !strcmp(getenv("SPLINTER_EMBEDDINGS"), "0"))) ? 128 : 3200;
  const size_t arena = slots * len, total = 5440 + slots * stride + arena;
  printf("Initializing store: %s\n", store.c_str());
  printf(" - Slots: %lu (%lu bytes each, %zu byte alignment)\n", slots, len, (size_t)alignof(struct splinter_slot));
  printf(" - Value Arena: %zu bytes, SRS: %zu bytes (~%.2f MB)\n", arena, total, (double)total / 1048576.0);
  int err = 0;
  spl_store* s = spl_store_create(store.c_str(), slots, len, flags, &err);
  int rc = 0;
  if (!s) { errno = err; perror("splinter_create"); rc = -1; }
  else spl_store_close(s);
  if (!save.empty()) {
    splinter_close();
    U.connected = open_store(save) == 0;
  }
  return rc ? 1 : 0;
}

void json_str(const char* s, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': fputs("\\\"", stdout); break;
      case '\\': fputs("\\\\", stdout); break;
      case '\b': fputs("\\b", stdout); break;
      case '\f': fputs("\\f", stdout); break;
      case '\n': fputs("\\n", stdout); break;
      case '\r': fputs("\\r", stdout); break;
      case '\t': fputs("\\t", stdout); break;
      default:
        if (c < 0x20) printf("\\u%04x", c);
        else putchar(c);
    }
  }
}

int cmd_export(int argc, char** argv) {
  if (!need_store("export")) return 1;
  if (argc >= 2 && strcmp(argv[1], "json")) { fprintf(stderr, "export: unsupported format '%s'\n", argv[1]); return 1; }
  size_t max_lines = argc >= 3 ? (size_t)atol(argv[2]) : 0;
  splinter_header_snapshot_t h{};
  splinter_get_header_snapshot(&h);
  std::vector<char*> names(h.slots ? h.slots : 1);
  size_t n = 0;
  splinter_list(names.data(), names.size(), &n);
  std::vector<splinter_slot_snapshot_t> snaps;
  for (size_t i = 0; i < n && (!max_lines || snaps.size() < max_lines); ++i) {
    splinter_slot_snapshot_t s{};
    if (splinter_get_slot_snapshot(names[i], &s) == 0) snaps.push_back(s);
  }
  printf("{\n  \"store\": {\n    \"total_slots\": %u,\n    \"active_keys\": %zu\n  },\n  \"keys\": [\n", h.slots,
         snaps.size());
  std::vector<char> buf(h.max_val_sz + 1);
  for (size_t i = 0; i < snaps.size(); ++i) {
    auto& s = snaps[i];
    printf("    {\n      \"key\": \"");
    json_str(s.key, strnlen(s.key, SPLINTER_KEY_MAX));
    printf("\",\n      \"type\": \"%s\",\n      \"epoch\": %lu,\n", type_name(s.type_flag), (unsigned long)s.epoch);
    if (s.type_flag & SPL_SLOT_TYPE_VARTEXT) {
      printf("      \"value_length\": %u,\n", s.val_len);
      size_t got = 0;
      if (splinter_get(s.key, buf.data(), h.max_val_sz, &got) == 0) {
        printf("      \"value\": \"");
        json_str(buf.data(), got);
        printf("\"\n");
      } else {
        printf("      \"value\": null\n");
      }
    } else {
      printf("      \"value_length\": %u\n", s.val_len);
    }
    printf(i + 1 < snaps.size() ? "    },\n" : "    }\n");
  }
  printf("  ]\n}\n");
  return 0;
}

// Minimal JSON reader for `import` (the inverse of `export json`; the reference
// has export only, SURVEY §5 checkpoint/resume).
struct JVal {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  double num = 0;
  bool b = false;
  std::string str;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;
  const JVal* get(const char* k) const {
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct JParser {
  const char* p;
  const char* end;
  bool ok = true;
  void ws() { while (p < end && isspace((unsigned char)*p)) ++p; }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(end - p) >= n && !strncmp(p, s, n)) { p += n; return true; }
    return false;
  }
  std::string string() {
    std::string out;
    ++p;  // opening quote
    while (p < end && *p != '"') {
      if (*p == '\\' && p + 1 < end) {
        ++p;
        switch (*p) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            if (end - p < 5) { ok = false; return out; }
            unsigned cp = (unsigned)strtoul(std::string(p + 1, 4).c_str(), nullptr, 16);
            p += 4;
            if (cp < 0x80) out += (char)cp;
            else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
            else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
            break;
          }
          default: out += *p;
        }
        ++p;
      } else {
        out += *p++;
      }
    }
    if (p < end) ++p; else ok = false;
    return out;
  }
  JVal value() {
    JVal v;
    ws();
    if (p >= end) { ok = false; return v; }
    if (*p == '{') {
      v.kind = JVal::Obj;
      ++p;
      ws();
      if (p < end && *p == '}') { ++p; return v; }
      while (ok) {
        ws();
        if (p >= end || *p != '"') { ok = false; break; }
        std::string k = string();
        ws();
        if (p >= end || *p != ':') { ok = false; break; }
        ++p;
        v.obj.emplace_back(k, value());
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '}') { ++p; break; }
        ok = false;
      }
    } else if (*p == '[') {
      v.kind = JVal::Arr;
      ++p;
      ws();
      if (p < end && *p == ']') { ++p; return v; }
      while (ok) {
        v.arr.push_back(value());
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == ']') { ++p; break; }
        ok = false;
      }
    } else if (*p == '"') {
      v.kind = JVal::Str;
      v.str = string();
    } else if (lit("true")) { v.kind = JVal::Bool; v.b = true; }
    else if (lit("false")) { v.kind = JVal::Bool; }
    else if (lit("null")) { v.kind = JVal::Null; }
    else {
      char* e = nullptr;
      v.num = strtod(p, &e);
      if (e == p) ok = false;
      v.kind = JVal::Num;
      p = e;
    }
    return v;
  }
};

unsigned type_from_full_name(const std::string& s) {
  for (unsigned t = 1; t <= SPL_SLOT_TYPE_VARTEXT; t <<= 1)
    if (s == type_name(t)) return t;
  return 0;
}

int cmd_import(int argc, char** argv) {
  if (!need_store("import")) return 1;
  const char* file = argc >= 2 ? argv[1] : "-";
  FILE* f = strcmp(file, "-") ? fopen(file, "rb") : stdin;
  if (!f) { fprintf(stderr, "import: cannot open '%s': %s\n", file, strerror(errno)); return 1; }
  std::string text;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
  if (f != stdin) fclose(f);
  JParser jp{text.data(), text.data() + text.size()};
  JVal root = jp.value();
  const JVal* keys = root.get("keys");
  if (!jp.ok || !keys || keys->kind != JVal::Arr) { fprintf(stderr, "import: not an `export json` document\n"); return 1; }
  size_t done = 0, skipped = 0;
  for (const JVal& k : keys->arr) {
    const JVal* name = k.get("key");
    const JVal* val = k.get("value");
    if (!name || name->kind != JVal::Str || !val || val->kind != JVal::Str) { ++skipped; continue; }
    const std::string key = pkey(name->str.c_str());
    if (splinter_set(key.c_str(), val->str.data(), val->str.size()) != 0) {
      fprintf(stderr, "import: set '%s' failed: %s\n", key.c_str(), strerror(errno));
      return 1;
    }
    if (const JVal* t = k.get("type"))
      if (unsigned tm = t->kind == JVal::Str ? type_from_full_name(t->str) : 0)
        splinter_set_named_type(key.c_str(), (uint16_t)tm);
    ++done;
  }
  printf("imported %zu key(s), skipped %zu without a value\n", done, skipped);
  return 0;
}

int cmd_type(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "Usage: type <key_name> [type]\n"); return 1; }
  if (!need_store("type")) return 1;
  std::string key = pkey(argv[1]);
  if (argc == 2) {
    splinter_slot_snapshot_t s{};
    if (splinter_get_slot_snapshot(key.c_str(), &s) != 0) { fprintf(stderr, "type: invalid key '%s'\n", key.c_str()); return 1; }
    printf("%s:%s\n", type_name(s.type_flag), key.c_str());
    puts("");
    return 0;
  }
  unsigned m = type_from_name(argv[2]);
  if (!m) { fprintf(stderr, "type: invalid bitmask alias: '%s'\n", argv[2]); return 1; }
  return splinter_set_named_type(key.c_str(), (uint16_t)m) == 0 ? 0 : 1;
}

int cmd_math(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "Usage: math <key> <op> [value]\n"); return 1; }
  if (!need_store("math")) return 1;
  std::string key = pkey(argv[1]);
  const char* op = argv[2];
  splinter_integer_op_t o;
  if (!strcasecmp(op, "inc")) o = SPL_OP_INC;
  else if (!strcasecmp(op, "dec")) o = SPL_OP_DEC;
  else if (!strcasecmp(op, "and")) o = SPL_OP_AND;
  else if (!strcasecmp(op, "or")) o = SPL_OP_OR;
  else if (!strcasecmp(op, "xor")) o = SPL_OP_XOR;
  else if (!strcasecmp(op, "not")) o = SPL_OP_NOT;
  else { fprintf(stderr, "math: unknown operation '%s'\n", op); return 1; }
  uint64_t v = 0;
  if (o != SPL_OP_NOT) {
    if (argc < 4) { fprintf(stderr, "math: operation '%s' requires a value\n", op); return 1; }
    if (!parse_mask(argv[3], &v)) { fprintf(stderr, "math: invalid value or label '%s'\n", argv[3]); return 1; }
  }
  if (splinter_integer_op(key.c_str(), o, &v) == 0) {
    printf("Operation '%s' applied to '%s' successfully.\n", op, key.c_str());
    return 0;
  }
  if (errno == EPROTOTYPE) fprintf(stderr, "math: key '%s' is not a BIGUINT slot.\n", key.c_str());
  else if (errno == EAGAIN) fprintf(stderr, "math: collision detected, try again.\n");
  else fprintf(stderr, "math: failed (errno: %d)\n", errno);
  return 1;
}

int cmd_label(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "Usage: label <key> <label_name|mask>   (prefix '-' removes)\n"); return 1; }
  if (!need_store("label")) return 1;
  std::string key = pkey(argv[1]);
  const char* lab = argv[2];
  bool remove = lab[0] == '-';
  uint64_t m;
  if (!parse_mask(remove ? lab + 1 : lab, &m)) { fprintf(stderr, "label: unknown label or invalid mask '%s'\n", lab); return 1; }
  int rc = remove ? splinter_unset_label(key.c_str(), m) : splinter_set_label(key.c_str(), m);
  if (rc == 0) {
    printf("Label '%s' (0x%lx) %s '%s'.\n", lab, (unsigned long)m, remove ? "removed from" : "applied to", key.c_str());
    return 0;
  }
  fprintf(stderr, "label: failed to apply label to '%s' (errno: %d)\n", key.c_str(), errno);
  return 1;
}

int cmd_orders(int argc, char** argv) {
  if (argc != 4) { fprintf(stderr, "Usage: orders <set|unset> <key> <count>\n"); return 1; }
  if (!need_store("orders")) return 1;
  std::string key = pkey(argv[2]);
  const int count = atoi(argv[3]);
  if (count < 1 || count > 255) { fprintf(stderr, "orders: count must be 1..255\n"); return 1; }
  if (!strcmp(argv[1], "set")) {
    std::vector<std::string> vals;
    std::vector<const void*> ptr;
    std::vector<size_t> lens;
    for (int i = 0; i < count; ++i) vals.push_back(std::string(SPL_ORDER_ACCESSOR) + "_" + std::to_string(i));
    for (auto& v : vals) { ptr.push_back(v.data()); lens.push_back(v.size()); }
    int r = splinter_client_set_tandem(key.c_str(), ptr.data(), lens.data(), (uint8_t)count);
    printf("Tandem set for %s with %d orders: %s\n", key.c_str(), count, r == 0 ? "OK" : "FAIL");
    return r ? 1 : 0;
  }
  if (!strcmp(argv[1], "unset")) {
    splinter_client_unset_tandem(key.c_str(), (uint8_t)count);
    printf("Tandem unset for %s (%d orders) executed.\n", key.c_str(), count);
    return 0;
  }
  fprintf(stderr, "Unsupported mode: %s ('set' or 'unset' are supported)\n", argv[1]);
  return 1;
}

int cmd_bind(int argc, char** argv) {
  std::vector<char*> pos;
  for (int i = 1; i < argc; ++i)
    if (strcmp(argv[i], "-b") && strcmp(argv[i], "--bloom")) pos.push_back(argv[i]);
  if (pos.size() != 2) { fprintf(stderr, "Usage: bind [label_name | mask] <group_id> [--bloom]\n"); return 1; }
  if (!need_store("bind")) return 1;
  uint64_t m;
  if (!parse_mask(pos[0], &m)) { fprintf(stderr, "bind: unknown label or invalid hex mask '%s'\n", pos[0]); return 1; }
  int g = atoi(pos[1]);
  if (g < 0 || g >= SPLINTER_MAX_GROUPS) { fprintf(stderr, "bind: invalid signal group '%d' (must be 0-63)\n", g); return 1; }
  if (splinter_watch_label_register(m, (uint8_t)g) == 0) {
    printf("Binding applied: Label '%s' (0x%lx) -> Signal Group %d\n", pos[0], (unsigned long)m, g);
    return 0;
  }
  fprintf(stderr, "bind: failed to register watch for mask 0x%lx (check store connection)\n", (unsigned long)m);
  return 1;
}

int cmd_bump(int argc, char** argv) {
  if (argc != 2) { fprintf(stderr, "Usage: bump <key_name>\n"); return 1; }
  if (!need_store("bump")) return 1;
  return splinter_bump_slot(pkey(argv[1]).c_str()) == 0 ? 0 : 1;
}

int cmd_append(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "Usage: append <key_name> \"<value_to_append>\"\n"); return 1; }
  if (!need_store("append")) return 1;
  size_t nl = 0;
  return splinter_append(pkey(argv[1]).c_str(), argv[2], strnlen(argv[2], 4096), &nl) == 0 ? 0 : 1;
}

int cmd_uuid(int, char**) {
  unsigned char b[16];
  int fd = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
  ssize_t r = fd >= 0 ? read(fd, b, 16) : -1;
  if (fd >= 0) close(fd);
  if (r != 16)
    for (int i = 0; i < 16; ++i) b[i] = (unsigned char)(rand() & 0xff);
  b[6] = (unsigned char)((b[6] & 0x0f) | 0x40);
  b[8] = (unsigned char)((b[8] & 0x3f) | 0x80);
  printf("%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x\n", b[0], b[1], b[2], b[3], b[4], b[5],
         b[6], b[7], b[8], b[9], b[10], b[11], b[12], b[13], b[14], b[15]);
  return 0;
}

int cmd_caps(int, char**) {
  printf("version=%s\n", SPLINTER_VERSION);
  printf("build=%s\n", SPL_BUILD_ID);
  printf("lua=yes (minilua, Lua 5.4 subset)\nwasm=yes (miniwasm, MVP interpreter)\nembeddings=yes\nllama=no\n");
#ifdef SYS_mbind
  {
    // mbind is compiled in; report whether the kernel has NUMA and how many nodes it exposes
    int nodes = 0;
    for (int n = 0; n < 1024; ++n) {
      char path[64];
      snprintf(path, sizeof path, "/sys/devices/system/node/node%d", n);
      if (access(path, F_OK) != 0) break;
      ++nodes;
    }
    if (nodes > 0) printf("numa=yes (%d node%s)\n", nodes, nodes == 1 ? "" : "s");
    else printf("numa=no (kernel without NUMA)\n");
  }
#else
  printf("numa=no (built without mbind)\n");
#endif
#ifdef SPLINTER_PERSISTENT
  printf("persistent=yes\n");
#else
  printf("persistent=%s\n", getenv("SPLINTER_PERSISTENT") ? "yes" : "no");
#endif
  printf("hbm=yes\ngfx=gfx950\nembedder=nomic-bert(hip)\n");
  return 0;
}

const char* intent_name(unsigned i) {
  switch (i) {
    case SPL_INTENT_WILLNEED: return "willneed";
    case SPL_INTENT_SEQUENTIAL: return "sequential";
    case SPL_INTENT_RANDOM: return "random";
    case SPL_INTENT_DONTNEED: return "dontneed";
    default: return "none";
  }
}
int intent_of(const char* s) {
  if (!strcmp(s, "willneed")) return SPL_INTENT_WILLNEED;
  if (!strcmp(s, "sequential")) return SPL_INTENT_SEQUENTIAL;
  if (!strcmp(s, "random")) return SPL_INTENT_RANDOM;
  if (!strcmp(s, "dontneed")) return SPL_INTENT_DONTNEED;
  if (!strcmp(s, "none")) return SPL_INTENT_NONE;
  return -1;
}

int cmd_shard(int argc, char** argv) {
  if (!need_store("shard")) return 1;
  const char* sub = argc >= 2 ? argv[1] : "table";
  if (!strcmp(sub, "table")) {
    splinter_shard_bid_snapshot t[SPLINTER_MAX_SHARDS];
    int n = splinter_shard_table_snapshot(t, SPLINTER_MAX_SHARDS);
    printf("%-4s %-10s %-8s %-11s %-4s %-20s %-20s %-7s %-9s\n", "slot", "shard_id", "pid", "intent", "prio",
           "claimed_at", "duration", "expired", "sovereign");
    for (int b = 0; b < n; ++b) {
      if (!t[b].shard_id) continue;
      printf("%-4d 0x%-8x %-8u %-11s %-4u %-20llu %-20llu %-7s %-9s\n", b, t[b].shard_id, t[b].pid,
             intent_name(t[b].intent), t[b].priority, (unsigned long long)t[b].claimed_at,
             (unsigned long long)t[b].duration_tsc, t[b].expired ? "yes" : "no", t[b].sovereign ? "yes" : "no");
    }
    return 0;
  }
  if (!strcmp(sub, "who")) {
    uint8_t it = 0;
    uint32_t id = splinter_shard_election(&it);
    if (!id) printf("no current sovereign\n");
    else printf("sovereign=0x%x intent=%s\n", id, intent_name(it));
    return 0;
  }
  if ((!strcmp(sub, "claim") || !strcmp(sub, "rebid")) && argc >= 6) {
    uint32_t id = (uint32_t)strtoul(argv[2], nullptr, 0);
    int it = intent_of(argv[3]);
    if (!id || it < 0) { fprintf(stderr, "shard: bad id or intent.\n"); return 1; }
    unsigned prio = (unsigned)strtoul(argv[4], nullptr, 0);
    unsigned long long dur = strtoull(argv[5], nullptr, 0);
    int rc = !strcmp(sub, "claim") ? splinter_shard_claim(id, (uint8_t)it, (uint8_t)prio, dur)
                                   : splinter_shard_rebid(id, (uint8_t)it, (uint8_t)prio, dur);
    if (rc) { fprintf(stderr, "shard %s failed (rc=%d, errno=%s)\n", sub, rc, strerror(errno)); return 1; }
    printf("%s 0x%x %s prio=%u dur=%llu OK\n", sub, id, intent_name((unsigned)it), prio, dur);
    return 0;
  }
  if (!strcmp(sub, "release") && argc >= 3) {
    uint32_t id = (uint32_t)strtoul(argv[2], nullptr, 0);
    int rc = splinter_shard_release(id);
    if (rc) { fprintf(stderr, "shard release failed (rc=%d): no such bid\n", rc); return 1; }
    printf("release 0x%x OK\n", id);
    return 0;
  }
  if (!strcmp(sub, "advise") && argc >= 4) {
    uint32_t id = (uint32_t)strtoul(argv[2], nullptr, 0);
    int it = intent_of(argv[3]);
    if (!id || it < 0) { fprintf(stderr, "shard: bad id or intent.\n"); return 1; }
    const int adv[] = {POSIX_MADV_NORMAL, POSIX_MADV_WILLNEED, POSIX_MADV_SEQUENTIAL, POSIX_MADV_RANDOM,
                       POSIX_MADV_DONTNEED};
    bool nowait = argc >= 5 && !strcmp(argv[4], "nowait");
    int rc = splinter_madvise(id, nullptr, 0, adv[it], nowait ? 0 : UINT64_MAX);
    if (rc) { fprintf(stderr, "shard advise: %s\n", strerror(errno)); return 1; }
    printf("advise 0x%x %s OK\n", id, intent_name((unsigned)it));
    return 0;
  }
  fprintf(stderr, "Usage: shard table|who|claim|rebid|release|advise ...\n");
  return 1;
}

int cmd_retrain(int argc, char** argv) {
  if (argc != 2) { fprintf(stderr, "Usage: retrain <key_name>\n"); return 1; }
  if (!need_store("retrain")) return 1;
  std::string key = pkey(argv[1]);
  if (splinter_retrain_slot(key.c_str()) != 0) {
    fprintf(stderr, "retrain: could not retrain '%s' (key not found?)\n", key.c_str());
    return 1;
  }
  return 0;
}

std::string slurp(FILE* f, size_t cap) {
  std::string s;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
  if (s.size() > cap) s.resize(cap);
  return s;
}

struct Hit {
  std::string key;
  float sim, dist;
  bool emb;
  uint64_t epoch, bloom;
  uint32_t len;
  uint8_t type;
};

int cmd_search(int argc, char** argv) {
  static option lo[] = {{"json", no_argument, nullptr, 'j'}, {"limit", required_argument, nullptr, 'L'},
                        {"distance", required_argument, nullptr, 'd'}, {"similarity", required_argument, nullptr, 's'},
                        {"bloom", required_argument, nullptr, 'B'}, {"regex", required_argument, nullptr, 'r'},
                        {"file", required_argument, nullptr, 'f'}, {"timeout", required_argument, nullptr, 't'},
                        {nullptr, 0, nullptr, 0}};
  bool json = false;
  int limit = 0, opt, timeout_ms = 2000;
  float max_dist = 0.f, min_sim = 0.f;
  uint64_t bloom = 0;
  const char *rx = nullptr, *file = nullptr;
  while ((opt = getopt_long(argc, argv, "jL:d:s:B:r:f:t:", lo, nullptr)) != -1) {
    switch (opt) {
      case 'j': json = true; break;
      case 'L': limit = atoi(optarg); break;
      case 'd': max_dist = strtof(optarg, nullptr); break;
      case 's': min_sim = strtof(optarg, nullptr); break;
      case 'B': parse_mask(optarg, &bloom); break;
      case 'r': rx = optarg; break;
      case 'f': file = optarg; break;
      case 't': timeout_ms = atoi(optarg); break;
      default: return 1;
    }
  }
  if (!need_store("search")) return 1;
  splinter_header_snapshot_t h{};
  splinter_get_header_snapshot(&h);
  std::string query;
  if (file) {
    FILE* f = strcmp(file, "-") ? fopen(file, "rb") : stdin;
    if (!f) { fprintf(stderr, "search: cannot open '%s': %s\n", file, strerror(errno)); return 1; }
    query = slurp(f, h.max_val_sz - 1);
    if (f != stdin) fclose(f);
  } else if (optind < argc) {
    query = !strcmp(argv[optind], "-") ? slurp(stdin, h.max_val_sz - 1) : argv[optind];
  }
  if (query.empty()) { fprintf(stderr, "Usage: search <query>|- [--file PATH] [--json] [--limit N] ...\n"); return 1; }
  // query embedding through the sidecar (reference cmd_search.c:301-326)
  std::string scratch = "__sqtmp_" + std::to_string(getpid());
  splinter_set(scratch.c_str(), query.data(), query.size());
  splinter_set_named_type(scratch.c_str(), SPL_SLOT_TYPE_VARTEXT);
  splinter_set_label(scratch.c_str(), 1ull);
  splinter_bump_slot(scratch.c_str());
  std::vector<float> q(SPLINTER_EMBED_DIM, 0.f);
  bool have_q = false;
  // wait for splinference's +2 epoch (set_embedding) after our bump
  auto t0 = std::chrono::steady_clock::now();
  uint64_t e0 = splinter_get_epoch(scratch.c_str());
  while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(timeout_ms)) {
    uint64_t e = splinter_get_epoch(scratch.c_str());
    if (!(e & 1) && e != e0 && splinter_get_embedding(scratch.c_str(), q.data()) == 0) {
      double m = 0;
      for (float v : q) m += (double)v * v;
      if (m > 1e-12) { have_q = true; break; }
    }
    usleep(2000);
  }
  if (!have_q) fprintf(stderr, "search: warning: splinference timed out; embedding scoring unavailable.\n");
  if (!have_q && !rx && !bloom) {
    fprintf(stderr, "search: splinference unavailable and no regex/bloom filter; no results.\n");
    splinter_unset(scratch.c_str());
    return 1;
  }
  regex_t re;
  bool filt = rx && regcomp(&re, rx, REG_EXTENDED | REG_NOSUB) == 0;
  std::vector<Hit> hits;
  // HBM store (or a node store of HBM shards: every GPU scores its shard, best hits merged): score
  // every candidate on the device (spl_hbm_search, libsplinter_hip.so K7 pass) instead of one slot
  // snapshot per candidate -- same candidates, filters and ranking.  A node of host shards makes
  // spl_hbm_search fail and takes the host path below.
  using HbmSearch = long (*)(spl_store*, const float*, uint64_t, float, float, long, spl_search_hit*);
  spl_store* cur = spl_store_current();
  HbmSearch gpu = nullptr;
  if (have_q && cur && (!strcmp(spl_store_backend(cur), "hbm") || !strcmp(spl_store_backend(cur), "node")))
    gpu = (HbmSearch)dlsym(RTLD_DEFAULT, "spl_hbm_search");
  bool done = false;
  if (gpu) {
    const long cap = (limit > 0 && !filt) ? limit + 1 : (long)h.slots;  // +1: our own scratch key
    std::vector<spl_search_hit> out((size_t)std::max<long>(cap, 1));
    const long n = gpu(cur, q.data(), bloom, min_sim, max_dist, cap, out.data());
    if (n >= 0) {
      for (long i = 0; i < std::min(n, cap); ++i) {
        const spl_search_hit& r = out[(size_t)i];
        std::string k(r.key);
        if (k == scratch) continue;
        if (filt && regexec(&re, k.c_str(), 0, nullptr, 0) != 0) continue;
        hits.push_back(Hit{k, r.sim, r.dist, r.emb != 0, r.epoch, r.bloom, r.len, r.type});
      }
      done = true;
    }
  }
  std::vector<std::string> cand;
  if (done) {
  } else if (bloom) {
    splinter_enumerate_matches(bloom, [](const char* k, uint64_t, void* ud) {
      ((std::vector<std::string>*)ud)->push_back(k);
    }, &cand);
  } else {
    std::vector<char*> names(h.slots ? h.slots : 1);
    size_t n = 0;
    splinter_list(names.data(), names.size(), &n);
    for (size_t i = 0; i < n; ++i) cand.push_back(names[i]);
  }
  double qn = 0;
  for (float v : q) qn += (double)v * v;
  qn = std::sqrt(qn);
  std::vector<float> v(SPLINTER_EMBED_DIM);
  for (auto& k : cand) {
    if (k == scratch) continue;
    if (filt && regexec(&re, k.c_str(), 0, nullptr, 0) != 0) continue;
    splinter_slot_snapshot_t s{};
    if (splinter_get_slot_snapshot(k.c_str(), &s) != 0) continue;
    Hit hit{k, 0.f, 0.f, false, s.epoch, s.bloom, s.val_len, s.type_flag};
    double vn = 0;
    for (int i = 0; i < SPLINTER_EMBED_DIM; ++i) vn += (double)s.embedding[i] * s.embedding[i];
    if (have_q && vn > 1e-12) {
      double dot = 0, d2 = 0;
      for (int i = 0; i < SPLINTER_EMBED_DIM; ++i) {
        dot += (double)s.embedding[i] * q[i];
        double d = (double)s.embedding[i] - q[i];
        d2 += d * d;
      }
      hit.sim = (float)(dot / (std::sqrt(vn) * qn));
      hit.dist = (float)std::sqrt(d2);
      hit.emb = true;
      if (min_sim > 0.f && hit.sim < min_sim) continue;
      if (max_dist > 0.f && hit.dist > max_dist) continue;
    } else if (min_sim > 0.f || max_dist > 0.f) {
      continue;
    }
    hits.push_back(hit);
  }
  if (filt) regfree(&re);
  std::sort(hits.begin(), hits.end(), [](const Hit& a, const Hit& b) {
    if (a.sim != b.sim) return a.sim > b.sim;
    return a.dist < b.dist;
  });
  size_t pc = hits.size();
  if (limit > 0 && pc > (size_t)limit) pc = (size_t)limit;
  if (json) {
    printf("{\n  \"query\": \"");
    json_str(query.data(), query.size());
    printf("\",\n  \"store\": {\n    \"total_slots\": %u,\n    \"active_keys\": %zu\n  },\n  \"results\": [\n", h.slots,
           hits.size());
    for (size_t i = 0; i < pc; ++i) {
      auto& r = hits[i];
      printf("    {\n      \"key\": \"");
      json_str(r.key.data(), r.key.size());
      printf("\",\n");
      if (r.emb) printf("      \"similarity\": %.4f,\n      \"distance\": %.4f,\n", r.sim, r.dist);
      else printf("      \"similarity\": null,\n      \"distance\": null,\n");
      printf("      \"epoch\": %lu,\n      \"value_length\": %u,\n      \"type\": \"%s\",\n", (unsigned long)r.epoch,
             r.len, type_name(r.type));
      printf("      \"bloom\": \"0x%016llx\",\n      \"has_embedding\": %s\n", (unsigned long long)r.bloom,
             r.emb ? "true" : "false");
      printf(i + 1 < pc ? "    },\n" : "    }\n");
    }
    printf("  ]\n}\n");
  } else {
    printf("%-44s %-10s %-10s %-6s %-6s %s\n", "Name", "Similarity", "Distance", "Epoch", "Len", "Type");
    for (size_t i = 0; i < pc; ++i) {
      auto& r = hits[i];
      if (r.emb)
        printf("%-44s %-10.4f %-10.4f %-6lu %-6u %s\n", r.key.c_str(), r.sim, r.dist, (unsigned long)r.epoch, r.len,
               type_name(r.type));
      else
        printf("%-44s %-10s %-10s %-6lu %-6u %s\n", r.key.c_str(), "-", "-", (unsigned long)r.epoch, r.len,
               type_name(r.type));
    }
    puts("");
  }
  splinter_unset(scratch.c_str());
  return 0;
}

int cmd_ingest(int argc, char** argv) {
  static option lo[] = {{"key", required_argument, nullptr, 'k'}, {"label", required_argument, nullptr, 'l'},
                        {"help", no_argument, nullptr, 'h'}, {nullptr, 0, nullptr, 0}};
  const uint64_t kChunkLabel = 0x200, kMetaLabel = 0x400;
  std::string key;
  uint64_t label = kChunkLabel;
  int opt;
  while ((opt = getopt_long(argc, argv, "k:l:h", lo, nullptr)) != -1) {
    if (opt == 'k') key = optarg;
    else if (opt == 'l') {
      if (!parse_mask(optarg, &label)) { fprintf(stderr, "ingest: invalid label '%s'\n", optarg); return 1; }
    } else return 1;
  }
  const char* file = optind < argc ? argv[optind] : nullptr;
  if (!file && key.empty()) { fprintf(stderr, "ingest: stdin input requires --key <name>\n"); return 1; }
  if (key.empty()) { std::string f(file); key = basename(&f[0]); }
  if (key.size() > 56) key.resize(56);
  key = U.prefix + key;
  if (!need_store("ingest")) return 1;
  FILE* fp = file ? fopen(file, "rb") : stdin;
  if (!fp) { fprintf(stderr, "ingest: cannot open '%s': %s\n", file, strerror(errno)); return 1; }
  splinter_header_snapshot_t h{};
  splinter_get_header_snapshot(&h);
  const size_t chunk = h.max_val_sz > 64 ? h.max_val_sz - 64 : h.max_val_sz;
  std::vector<char> buf(chunk);
  size_t nread, count = 0, total = 0;
  const char* src = file ? file : "(stdin)";
  printf("[ingest] key='%s' chunk_sz=%zu source='%s'\n", key.c_str(), chunk, src);
  int rc = 0;
  while ((nread = fread(buf.data(), 1, chunk, fp)) > 0) {
    ++count;
    total += nread;
    std::string k = key + SPL_ORDER_ACCESSOR + std::to_string(count);
    if (splinter_set(k.c_str(), buf.data(), nread) != 0) {
      fprintf(stderr, "ingest: failed to write chunk %zu ('%s')\n", count, k.c_str());
      rc = 1;
      break;
    }
    splinter_set_named_type(k.c_str(), SPL_SLOT_TYPE_VARTEXT);
    splinter_set_label(k.c_str(), label);
    splinter_bump_slot(k.c_str());
    printf("[ingest] chunk %zu: %zu bytes\n", count, nread);
  }
  if (fp != stdin) fclose(fp);
  if (!rc && count == 0) { fprintf(stderr, "ingest: input was empty, nothing ingested\n"); return 1; }
  if (!rc) {
    char meta[512];
    int n = snprintf(meta, sizeof meta, "{\"chunks\":%zu,\"bytes\":%zu,\"source\":\"%s\",\"ingested\":%ld}", count,
                     total, src, (long)time(nullptr));
    if (splinter_set(key.c_str(), meta, (size_t)n) != 0) { fprintf(stderr, "ingest: failed to write metadata slot '%s'\n", key.c_str()); return 1; }
    splinter_set_named_type(key.c_str(), SPL_SLOT_TYPE_JSON);
    splinter_set_label(key.c_str(), kMetaLabel);
    printf("[ingest] done: %zu chunk(s), %zu bytes total -> '%s'\n", count, total, key.c_str());
  }
  return rc;
}

int cmd_stats(int, char**) {
  if (!need_store("stats")) return 1;
  splinter_header_snapshot_t h{};
  splinter_get_header_snapshot(&h);
  std::vector<char*> names(h.slots ? h.slots : 1);
  size_t n = 0;
  splinter_list(names.data(), names.size(), &n);
  size_t embedded = 0;
  std::vector<float> v(SPLINTER_EMBED_DIM);
  for (size_t i = 0; i < n; ++i)
    if (splinter_get_embedding(names[i], v.data()) == 0) {
      double m = 0;
      for (float x : v) m += (double)x * x;
      embedded += m > 1e-12;
    }
  printf("backend=%s\nslots=%u\nmax_val=%u\nactive_keys=%zu\nload=%.4f\nembedded=%zu\nepoch=%lu\nmop=%d\n",
         spl_store_backend(spl_store_current()), h.slots, h.max_val_sz, n, h.slots ? (double)n / h.slots : 0.0, embedded,
         (unsigned long)h.epoch, splinter_get_mop());
  for (int g = 0; g < SPLINTER_MAX_GROUPS; ++g) {
    uint64_t c = splinter_get_signal_count((uint8_t)g);
    if (c) printf("signal_group[%d]=%lu\n", g, (unsigned long)c);
  }
  // probe-chain health of an hbm: / node: store (libsplinter_hip.so, one device pass): how far a hit
  // and a miss probe, and the tombstones that make misses walk further
  using ProbeFn = int (*)(spl_store*, spl_probe_stats*);
  auto probe = (ProbeFn)dlsym(RTLD_DEFAULT, "spl_hbm_probe_stats");
  spl_probe_stats ps{};
  if (probe && probe(spl_store_current(), &ps) == 0) {
    const double homes = (double)h.slots;
    printf("probe_live=%lu\nprobe_tombstones=%lu\nprobe_virgin=%lu\nprobe_busy=%lu\n", (unsigned long)ps.live,
           (unsigned long)ps.tombstones, (unsigned long)ps.virgin, (unsigned long)ps.busy);
    printf("probe_hit_mean=%.3f\nprobe_hit_max=%lu\n", ps.live ? (double)ps.disp_sum / ps.live : 0.0,
           (unsigned long)ps.disp_max);
    if (ps.virgin)
      printf("probe_miss_mean=%.3f\nprobe_miss_max=%lu\n", homes ? (double)ps.miss_sum / homes : 0.0,
             (unsigned long)ps.miss_max);
    else
      printf("probe_miss_mean=%u\nprobe_miss_max=%u\n", h.slots, h.slots);  // no never-used slot: a miss scans all
    static const char* lab[12] = {"1", "2", "3-4", "5-8", "9-16", "17-32", "33-64", "65-128", "129-256", "257-512",
                                  "513-1024", ">1024"};
    for (int b = 0; b < 12; ++b)
      if (ps.hist[b]) printf("probe_hist[%s]=%lu\n", lab[b], (unsigned long)ps.hist[b]);
    printf("rehash_runs=%lu\nrehash_moved=%lu\nrehash_reclaimed=%lu\n", (unsigned long)ps.rebuilds,
           (unsigned long)ps.moved, (unsigned long)ps.reclaimed);
  }
  return 0;
}

// `rehash [--full]`: tombstone maintenance of an hbm: / node: store (spl_hbm_rehash_ex): the online
// compaction by default (safe beside live clients), --full the exclusive rebuild
int cmd_rehash(int argc, char** argv) {
  if (!need_store("rehash")) return 1;
  unsigned flags = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--full")) flags |= 1u;  // SPL_REHASH_FULL
    else {
      fprintf(stderr, "rehash: unknown option %s\n", argv[i]);
      return 1;
    }
  }
  using RehashFn = int (*)(spl_store*, unsigned, uint64_t*);
  auto fn = (RehashFn)dlsym(RTLD_DEFAULT, "spl_hbm_rehash_ex");
  uint64_t out[4] = {0, 0, 0, 0};
  errno = 0;
  if (!fn || fn(spl_store_current(), flags, out) != 0) {
    if (errno == EBUSY)
      fprintf(stderr, "rehash: busy (another maintenance pass is running%s)\n",
              flags ? ", or this store's ring worker could not be held" : "");
    else if (errno == ENOMEM)
      fprintf(stderr, "rehash: the full rebuild's scratch does not fit on the device; run the online rehash\n");
    else
      fprintf(stderr, "rehash: only hbm: and node: stores of HBM shards (device pass), or the pass failed\n");
    return 1;
  }
  printf("moved=%lu\nreclaimed=%lu\nclusters=%lu\nskipped=%lu\n", (unsigned long)out[0], (unsigned long)out[1],
         (unsigned long)out[2], (unsigned long)out[3]);
  return 0;
}

// `lua` verb: the reference's `splinter` Lua module (splinter_cli_cmd_lua.c:
// 20-360) bound to the current store, run on minilua.
mlua::Value splinter_module() {
  using mlua::Value;
  using mlua::Values;
  auto T = std::make_shared<mlua::Table>();
  auto str = [](Values& a, size_t i, const char* fn) -> std::string {
    if (i < a.size() && a[i].t == Value::Str) return *a[i].s;
    if (i < a.size() && a[i].is_num()) return mlua::tostring(a[i]);
    throw mlua::LuaError(std::string("bad argument #") + std::to_string(i + 1) + " to '" + fn + "' (string expected)");
  };
  auto integer = [](Values& a, size_t i, int64_t dflt) -> int64_t {
    if (i >= a.size() || a[i].t == Value::Nil) return dflt;
    if (a[i].t == Value::Int) return a[i].i;
    if (a[i].t == Value::Num) return (int64_t)a[i].n;
    if (a[i].t == Value::Str) return (int64_t)strtoll(a[i].s->c_str(), nullptr, 0);
    throw mlua::LuaError("number expected");
  };
  auto reg = [&](const char* n, mlua::Native f) { T->set(Value::string(n), mlua::make_native(n, std::move(f))); };
  reg("get", [str](mlua::Interp&, Values& a) {
    const std::string key = pkey(str(a, 0, "get").c_str());
    splinter_header_snapshot_t h{};
    splinter_get_header_snapshot(&h);
    std::vector<char> buf(h.max_val_sz + 8);
    size_t n = 0;
    if (splinter_get(key.c_str(), buf.data(), buf.size(), &n) != 0) return Values{Value()};
    splinter_slot_snapshot_t snap{};
    if (splinter_get_slot_snapshot(key.c_str(), &snap) == 0 && (snap.type_flag & SPL_SLOT_TYPE_BIGUINT) && n >= 8) {
      uint64_t v;
      memcpy(&v, buf.data(), 8);
      return Values{Value::integer((int64_t)v)};
    }
    return Values{Value::string(std::string(buf.data(), n))};
  });
  reg("get_tandem", [str, integer](mlua::Interp&, Values& a) {
    const std::string base = pkey(str(a, 0, "get_tandem").c_str());
    const int64_t max_orders = integer(a, 1, 64);
    splinter_header_snapshot_t h{};
    splinter_get_header_snapshot(&h);
    std::vector<char> buf(h.max_val_sz + 8);
    auto t = std::make_shared<mlua::Table>();
    for (int64_t i = 0; i < max_orders; ++i) {
      const std::string k = i == 0 ? base : base + SPL_ORDER_ACCESSOR + std::to_string(i);
      size_t n = 0;
      if (splinter_get(k.c_str(), buf.data(), buf.size(), &n) != 0) break;
      t->set(Value::integer(i + 1), Value::string(std::string(buf.data(), n)));
    }
    return Values{Value::table(t)};
  });
  reg("set", [str](mlua::Interp&, Values& a) {
    const std::string key = pkey(str(a, 0, "set").c_str());
    if (a.size() > 1 && a[1].is_num()) {  // numbers become BIGUINT slots (reference :171-199)
      uint64_t v = (uint64_t)(a[1].t == Value::Int ? a[1].i : (int64_t)a[1].n);
      if (splinter_set(key.c_str(), &v, 8) != 0) return Values{Value::boolean(false)};
      splinter_set_named_type(key.c_str(), SPL_SLOT_TYPE_BIGUINT);
      return Values{Value::boolean(true)};
    }
    const std::string v = str(a, 1, "set");
    return Values{Value::boolean(splinter_set(key.c_str(), v.data(), v.size()) == 0)};
  });
  reg("set_tandem", [str](mlua::Interp&, Values& a) {
    const std::string base = pkey(str(a, 0, "set_tandem").c_str());
    if (a.size() < 2 || a[1].t != Value::Tab) throw mlua::LuaError("bad argument #2 to 'set_tandem' (table expected)");
    const int64_t n = a[1].tab->length();
    for (int64_t i = 1; i <= n; ++i) {
      const std::string k = i == 1 ? base : base + SPL_ORDER_ACCESSOR + std::to_string(i - 1);
      const std::string v = mlua::tostring(a[1].tab->get(Value::integer(i)));
      if (splinter_set(k.c_str(), v.data(), v.size()) != 0) return Values{Value::boolean(false)};
    }
    return Values{Value::boolean(true)};
  });
  reg("math", [str, integer](mlua::Interp&, Values& a) {
    const std::string key = pkey(str(a, 0, "math").c_str()), op = str(a, 1, "math");
    uint64_t v = (uint64_t)integer(a, 2, 0);
    splinter_integer_op_t o;
    if (op == "and") o = SPL_OP_AND;
    else if (op == "or") o = SPL_OP_OR;
    else if (op == "xor") o = SPL_OP_XOR;
    else if (op == "not") o = SPL_OP_NOT;
    else if (op == "inc") o = SPL_OP_INC;
    else if (op == "dec") o = SPL_OP_DEC;
    else throw mlua::LuaError("invalid math operation: " + op);
    if (splinter_integer_op(key.c_str(), o, &v) == 0) return Values{Value::boolean(true)};
    if (errno == EPROTOTYPE) throw mlua::LuaError("key '" + key + "' is not a BIGUINT slot");
    return Values{Value::boolean(false)};
  });
  reg("watch", [str, integer](mlua::Interp&, Values& a) {
    return Values{Value::boolean(splinter_watch_register(pkey(str(a, 0, "watch").c_str()).c_str(),
                                                         (uint8_t)integer(a, 1, 0)) == 0)};
  });
  reg("unwatch", [str, integer](mlua::Interp&, Values& a) {
    return Values{Value::boolean(splinter_watch_unregister(pkey(str(a, 0, "unwatch").c_str()).c_str(),
                                                           (uint8_t)integer(a, 1, 0)) == 0)};
  });
  reg("label", [str](mlua::Interp&, Values& a) {
    if (a.size() < 2 || !a[1].is_num()) throw mlua::LuaError("Label must be a numeric mask");
    const uint64_t m = (uint64_t)(a[1].t == Value::Int ? a[1].i : (int64_t)a[1].n);
    return Values{Value::boolean(splinter_set_label(pkey(str(a, 0, "label").c_str()).c_str(), m) == 0)};
  });
  reg("unset", [str](mlua::Interp&, Values& a) {
    const int r = splinter_unset(pkey(str(a, 0, "unset").c_str()).c_str());
    return Values{r >= 0 ? Value::integer(r) : Value::boolean(false)};
  });
  reg("bump", [str](mlua::Interp&, Values& a) {
    return Values{Value::boolean(splinter_bump_slot(pkey(str(a, 0, "bump").c_str()).c_str()) == 0)};
  });
  reg("sleep", [integer](mlua::Interp&, Values& a) {
    int64_t ms = integer(a, 0, 0);
    if (ms > 0) usleep((useconds_t)ms * 1000);
    return Values{};
  });
  reg("get_embedding", [str](mlua::Interp&, Values& a) {
    std::vector<float> v(SPLINTER_EMBED_DIM);
    if (splinter_get_embedding(pkey(str(a, 0, "get_embedding").c_str()).c_str(), v.data()) != 0) return Values{Value()};
    double m = 0;
    for (float x : v) m += (double)x * x;
    if (std::sqrt(m) <= 1e-6) return Values{Value()};
    auto t = std::make_shared<mlua::Table>();
    for (int i = 0; i < SPLINTER_EMBED_DIM; ++i) t->set(Value::integer(i + 1), Value::number(v[(size_t)i]));
    return Values{Value::table(t)};
  });
  reg("set_embedding", [str](mlua::Interp&, Values& a) {
    if (a.size() < 2 || a[1].t != Value::Tab) throw mlua::LuaError("bad argument #2 to 'set_embedding' (table expected)");
    const int64_t n = a[1].tab->length();
    if (n != SPLINTER_EMBED_DIM)
      throw mlua::LuaError("embedding table must hold exactly " + std::to_string(SPLINTER_EMBED_DIM) + " floats (got " +
                           std::to_string(n) + ")");
    std::vector<float> v(SPLINTER_EMBED_DIM);
    for (int i = 0; i < SPLINTER_EMBED_DIM; ++i) {
      Value x = a[1].tab->get(Value::integer(i + 1));
      if (!x.is_num()) throw mlua::LuaError("embedding element " + std::to_string(i + 1) + " is not a number");
      v[(size_t)i] = (float)x.as_double();
    }
    return Values{Value::boolean(splinter_set_embedding(pkey(str(a, 0, "set_embedding").c_str()).c_str(), v.data()) == 0)};
  });
  return Value::table(T);
}

int cmd_lua(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "Usage: lua <script.lua> [args...]\n"); return 1; }
  if (!need_store("lua")) return 1;
  FILE* f = fopen(argv[1], "rb");
  if (!f) { fprintf(stderr, "lua: cannot open '%s': %s\n", argv[1], strerror(errno)); return 1; }
  std::string src;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) src.append(buf, n);
  fclose(f);
  mlua::Interp I;
  I.out = [](const std::string& s) { fwrite(s.data(), 1, s.size(), stdout); fflush(stdout); };
  mlua::Value mod = splinter_module();
  I.modules["splinter"] = mod;
  I.set_global("splinter", mod);
  std::vector<std::string> args;
  for (int i = 2; i < argc; ++i) args.push_back(argv[i]);
  try {
    I.run(src, argv[1], args);
  } catch (const mlua::LuaError& e) {
    fprintf(stderr, "lua: %s\n", e.what());
    return 1;
  }
  return 0;
}

// `wasm` verb: the reference's WasmEdge host module (splinter_cli_cmd_wasm.c:
// 20-77, 85-143) on the built-in interpreter.  Host functions of module
// "splinter" (guest pointers/lengths are i32 into exported memory 0):
//   set(key_ptr, key_len, val_ptr, val_len) -> i32   1 on success, 0 on failure (as the reference)
//   get(key_ptr, key_len, out_ptr) -> i32            value length copied to out_ptr, -1 if absent
//                                                    (the reference's get is a stub returning 0)
//   unset(key_ptr, key_len) -> i32                   bytes freed, -1 if absent
//   print(ptr, len)                                  writes guest bytes to stdout
int cmd_wasm(int argc, char** argv) {
  if (argc < 2) { puts("Usage: wasm <plugin.wasm|plugin.wat> [function_name]"); return 1; }
  if (!need_store("wasm")) return 1;
  const char* path = argv[1];
  const std::string fn = argc > 2 ? argv[2] : "_start";
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "WASM Execution failed: cannot open '%s': %s\n", path, strerror(errno)); return 1; }
  std::vector<uint8_t> bytes;
  uint8_t buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) bytes.insert(bytes.end(), buf, buf + n);
  fclose(f);
  using mwasm::FuncType;
  using mwasm::I32;
  auto key_of = [](mwasm::Instance& in, uint64_t p, uint64_t len) {
    const uint64_t l = len < SPLINTER_KEY_MAX ? len : SPLINTER_KEY_MAX - 1;
    return std::string((const char*)in.mem_ptr((uint32_t)p, (uint32_t)l), (size_t)l);
  };
  std::map<std::string, std::pair<FuncType, mwasm::HostFn>> hosts;
  hosts["splinter.set"] = {FuncType{{I32, I32, I32, I32}, {I32}}, [&](mwasm::Instance& in, const uint64_t* a, uint64_t* r) {
    const std::string k = key_of(in, a[0], a[1]);
    const uint8_t* v = in.mem_ptr((uint32_t)a[2], (uint32_t)a[3]);
    r[0] = splinter_set(k.c_str(), v, (size_t)(uint32_t)a[3]) == 0 ? 1 : 0;
  }};
  hosts["splinter.get"] = {FuncType{{I32, I32, I32}, {I32}}, [&](mwasm::Instance& in, const uint64_t* a, uint64_t* r) {
    const std::string k = key_of(in, a[0], a[1]);
    splinter_header_snapshot_t hs{};
    splinter_get_header_snapshot(&hs);
    std::vector<uint8_t> v((size_t)hs.max_val_sz + 1);
    size_t len = 0;
    if (splinter_get(k.c_str(), v.data(), v.size(), &len) != 0) { r[0] = (uint32_t)-1; return; }
    memcpy(in.mem_ptr((uint32_t)a[2], len), v.data(), len);
    r[0] = (uint32_t)len;
  }};
  hosts["splinter.unset"] = {FuncType{{I32, I32}, {I32}}, [&](mwasm::Instance& in, const uint64_t* a, uint64_t* r) {
    r[0] = (uint32_t)splinter_unset(key_of(in, a[0], a[1]).c_str());
  }};
  hosts["splinter.print"] = {FuncType{{I32, I32}, {}}, [&](mwasm::Instance& in, const uint64_t* a, uint64_t*) {
    fwrite(in.mem_ptr((uint32_t)a[0], (uint32_t)a[1]), 1, (size_t)(uint32_t)a[1], stdout);
    fflush(stdout);
  }};
  try {
    mwasm::Instance inst(mwasm::parse_any(bytes), hosts);
    inst.step_limit = 1ull << 34;
    if (!inst.export_type(fn).params.empty()) throw mwasm::Error("function '" + fn + "' takes arguments");
    inst.invoke(fn);
  } catch (const mwasm::Error& e) {
    fprintf(stderr, "WASM Execution failed: %s\n", e.what());
    return 1;
  }
  return 0;
}


void register_modules() {
  auto& m = modules();
  m = {
      {"clear", "Clears the screen.", cmd_clear, nullptr},
      {"cls", "Alias of 'clear'", cmd_clear, nullptr},
      {"config", "Access Splinter bus and slot metadata.", cmd_config,
       [] { puts("Usage: config\n       config av <0|1|2>   (mop: 0 off, 1 hybrid, 2 full)"); }},
      {"get", "Retrieve the value of a key in the store.", cmd_get, [] { puts("Usage: get <key_name>"); }},
      {"head", "Retrieve just the metadata of a key in the store.", cmd_head, [] { puts("Usage: head <key_name>"); }},
      {"help", "Help with commands and features.", cmd_help, [] { puts("Usage: help [ext] [command]"); }},
      {"hist", "View and clear command history.", cmd_hist, [] { puts("Usage: hist [pattern] | hist clear"); }},
      {"list", "List keys in the current store.", cmd_list, [] { puts("Usage: list [pattern] [max_lines]"); }},
      {"set", "Set a key in the store to a specified value.", cmd_set, [] { puts("Usage: set <key> <value>"); }},
      {"unset", "Delete a key from the store.", cmd_unset, [] { puts("Usage: unset [-r] <key_name>"); }},
      {"use", "Switch to a different store.", cmd_use, [] { puts("Usage: use <store | file path | hbm:name>"); }},
      {"watch", "Watch a key or signal group for changes.", cmd_watch,
       [] { puts("Usage: watch <key> [--oneshot]\n       watch --group <id> [--oneshot]"); }},
      {"init", "Initialize a new store.", cmd_init,
       [] { puts("Usage: init [--slots N] [--length N] [--embeddings|--no-embeddings] [store]"); }},
      {"export", "Export the store to standard output.", cmd_export, [] { puts("Usage: export [json] [max_lines]"); }},
      {"import", "Import keys from an `export json` document.", cmd_import, [] { puts("Usage: import [file|-]"); }},
      {"type", "Display or set the named type of a key.", cmd_type,
       [] { puts("Usage: type <key> [void|bigint|biguint|json|binary|img|audio|vartext]"); }},
      {"math", "Atomic integer operations on BIGUINT keys.", cmd_math,
       [] { puts("Usage: math <key> <inc|dec|and|or|xor|not> [value|label]"); }},
      {"label", "Apply (or with '-' prefix remove) a bloom label.", cmd_label, [] { puts("Usage: label <key> <label|mask>"); }},
      {"orders", "Manage tandem (ordered) keys.", cmd_orders, [] { puts("Usage: orders <set|unset> <key> <count>"); }},
      {"bind", "Bind a bloom label to a signal group.", cmd_bind, [] { puts("Usage: bind <label|mask> <group_id>"); }},
      {"bump", "Advance a key's epoch (pulse watchers).", cmd_bump, [] { puts("Usage: bump <key_name>"); }},
      {"append", "Append to a key's value.", cmd_append, [] { puts("Usage: append <key_name> \"<value>\""); }},
      {"uuid", "Print a UUID v4.", cmd_uuid, nullptr},
      {"caps", "Print version, build and feature flags.", cmd_caps, nullptr},
      {"shard", "Inspect and seed the Logic Shard bid table.", cmd_shard,
       [] { puts("Usage: shard table|who|claim <id> <intent> <prio> <dur>|rebid ...|release <id>|advise <id> <intent> [nowait]"); }},
      {"retrain", "Zero a key's vector and rewind its epoch to 4.", cmd_retrain, [] { puts("Usage: retrain <key_name>"); }},
      {"search", "Semantic search over embedded keys.", cmd_search,
       [] { puts("Usage: search <query>|- [--file PATH] [--json] [--limit N] [--distance F] [--similarity F] [--bloom MASK] [--regex PATTERN]"); }},
      {"ingest", "Chunk a file or stdin into VARTEXT tandem keys.", cmd_ingest,
       [] { puts("Usage: ingest [file] [--key <key>] [--label <hex>]"); }},
      {"stats", "Store occupancy, embeddings, signal counters and (hbm/node) probe-chain health.", cmd_stats, nullptr},
      {"rehash", "Rebuild probe chains: move keys into tombstones on their path, reclaim trailing ones (hbm/node, online).",
       cmd_rehash, [] { puts("Usage: rehash [--full]   (online beside live clients; --full: exclusive rebuild, stop every client first)"); }},
      {"wasm", "Run a WASM module (binary or WAT) against the store.", cmd_wasm,
       [] { puts("Usage: wasm <plugin.wasm|plugin.wat> [function_name]\nExecutes a WASM module with access to the Splinter bus."); }},
      {"lua", "Run a Lua script against the store (splinter module).", cmd_lua,
       [] { puts("Usage: lua <script.lua> [args...]   (require(\"splinter\"): get get_tandem set set_tandem math\n"
                 "       watch unwatch label unset bump sleep get_embedding set_embedding)"); }},
  };
}

void on_signal(int) { U.abort = 1; }

}  // namespace

int main(int argc, char** argv) {
  register_modules();
  std::string prog = basename(argv[0]);
  bool repl = !(prog == "splinterctl" || prog == "splinterpctl");
  if (const char* p = getenv("SPLINTER_NS_PREFIX")) U.prefix = p;
  if (const char* h = getenv("SPLINTER_HISTORY_FILE")) U.history_file = h;
  if (const char* l = getenv("SPLINTER_HISTORY_LEN")) U.history_len = atoi(l);
  std::string rc_path, use = getenv("SPLINTER_DEFAULT_STORE") ? getenv("SPLINTER_DEFAULT_STORE") : "";
  static option lo[] = {{"help", optional_argument, nullptr, 'h'}, {"history-file", required_argument, nullptr, 'H'},
                        {"history-len", required_argument, nullptr, 'l'}, {"list-modules", no_argument, nullptr, 'L'},
                        {"no-repl", no_argument, nullptr, 'n'}, {"rc-file", required_argument, nullptr, 'r'},
                        {"prefix", required_argument, nullptr, 'p'}, {"use", required_argument, nullptr, 'u'},
                        {"version", no_argument, nullptr, 'v'}, {nullptr, 0, nullptr, 0}};
  int opt;
  while ((opt = getopt_long(argc, argv, "+h::H:l:Lnp:r:u:v", lo, nullptr)) != -1) {
    switch (opt) {
      case 'h': {
        std::vector<std::string> a{"help"};
        if (optarg) a.push_back(optarg);
        return run_argv(a);
      }
      case 'H': U.history_file = optarg; break;
      case 'l': U.history_len = atoi(optarg); break;
      case 'L':
        for (auto& m : modules()) printf("%s\n", m.name);
        return 0;
      case 'n': repl = false; break;
      case 'p': U.prefix = optarg; break;
      case 'r': rc_path = optarg; break;
      case 'u': use = optarg; break;
      case 'v': printf("%s %s (build %s)\n", prog.c_str(), SPLINTER_VERSION, SPL_BUILD_ID); return 0;
      default: return 1;
    }
  }
  load_rc(rc_path);
  if (use.empty()) use = DEFAULT_BUS;
  U.connected = open_store(use) == 0;
  if (!U.connected) U.store = use;
  signal(SIGUSR1, on_signal);
  signal(SIGUSR2, on_signal);
  if (!U.history_file.empty()) {
    FILE* f = fopen(U.history_file.c_str(), "r");
    char line[4096];
    while (f && fgets(line, sizeof line, f)) {
      line[strcspn(line, "\n")] = 0;
      U.history.push_back(line);
    }
    if (f) fclose(f);
  }
  int rc = 0;
  if (!repl) {
    std::vector<std::string> a;
    for (int i = optind; i < argc; ++i) a.push_back(argv[i]);
    if (a.empty()) {
      fprintf(stderr, "Usage: %s [options] <command> [args]\n", prog.c_str());
      return 1;
    }
    rc = run_argv(a);
  } else {
    signal(SIGINT, on_signal);
    fprintf(stderr, "%s %s (build %s)\nTo quit, press ctrl-c or ctrl-d.\n", prog.c_str(), SPLINTER_VERSION, SPL_BUILD_ID);
    std::string line;
    // Tab completes the command word, like the reference's linenoise callback
    const spl_le::Completer complete = [](const std::string& b, std::vector<std::string>& out) {
      if (b.find(' ') != std::string::npos) return;
      for (auto& m : modules())
        if (!strncmp(m.name, b.c_str(), b.size())) out.push_back(m.name);
    };
    for (;;) {
      std::string prompt = (rc ? std::to_string(rc) + " : " : std::string()) +
                           (U.connected ? U.store : std::string("no-conn")) + " # ";
      const spl_le::Read r = spl_le::read_line(prompt.c_str(), line, U.history, complete);
      if (r != spl_le::Read::Line) break;  // Ctrl-D / EOF, or Ctrl-C: quit as the banner says
      auto a = tokenize(line);
      if (a.empty()) continue;
      U.history.push_back(line);
      if ((int)U.history.size() > U.history_len) U.history.erase(U.history.begin());
      if (a[0] == "quit" || a[0] == "exit") break;
      U.abort = 0;
      rc = run_argv(a);
      fflush(stdout);
    }
  }
  if (!U.history_file.empty() && U.history_len > 0) {
    FILE* f = fopen(U.history_file.c_str(), "w");
    for (size_t i = 0; f && i < U.history.size(); ++i) fprintf(f, "%s\n", U.history[i].c_str());
    if (f) fclose(f);
  }
  splinter_close();
  return rc;
}
