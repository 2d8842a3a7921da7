// capi.cpp — reference-compatible C API (splinter_*) and the handle API
// (spl_*) over StoreBase.  Backend selection by store name:
//   "hbm:NAME"            -> HBM arena (libsplinter_hip.so, dlopen'd lazily)
//   "node:NAME"           -> one store over a node's per-GPU arenas (node_store.hpp)
//   "file:PATH" / a path  -> regular file (reference -DSPLINTER_PERSISTENT)
//   "shm:NAME" / NAME     -> POSIX shm object (reference default)
// Reference C API: /root/reference/splinter.h:288-1213.
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <mutex>
#include <poll.h>
#include <string>
#include <vector>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#define SPLINTER_NO_INLINE_NOW 1
#include "splinter_ext.h"
#include "node_store.hpp"
#include "store_host.hpp"

#ifndef SPL_BUILD_ID
#define SPL_BUILD_ID "dev"
#endif

using spl::StoreBase;

namespace {

std::atomic<StoreBase*> g_cur{nullptr};  // the reference's "one open store per process" (atomic: any thread may switch it)

enum class Kind { Shm, File, Hbm, Node };

struct Parsed {
  Kind kind;
  std::string name;
};

bool env_true(const char* v) { return v && *v && std::strcmp(v, "0") != 0; }

Parsed parse_name(const char* raw) {
  std::string s(raw ? raw : "");
  if (s.rfind("hbm:", 0) == 0) return {Kind::Hbm, s.substr(4)};
  if (s.rfind("node:", 0) == 0) return {Kind::Node, s.substr(5)};
  if (s.rfind("file:", 0) == 0) return {Kind::File, s.substr(5)};
  if (s.rfind("shm:", 0) == 0) return {Kind::Shm, s.substr(4)};
#ifdef SPLINTER_PERSISTENT
  return {Kind::File, s};
#else
  if (env_true(getenv("SPLINTER_PERSISTENT"))) return {Kind::File, s};
  // a '/' anywhere but the leading character means a filesystem path
  if (s.find('/', 1) != std::string::npos || s.rfind("./", 0) == 0) return {Kind::File, s};
  return {Kind::Shm, s};
#endif
}

std::mutex g_hbm_mu;
spl::HbmFactory g_hbm_factory = nullptr;
void* g_hip_handle = nullptr;

void* hip_handle_locked() {
  if (g_hip_handle) return g_hip_handle;
  std::string path;
  if (const char* env = getenv("SPLINTER_HIP_LIB")) {
    path = env;
  } else {
    Dl_info info;
    if (dladdr((void*)&hip_handle_locked, &info) && info.dli_fname) {
      std::string self(info.dli_fname);
      size_t slash = self.rfind('/');
      path = (slash == std::string::npos ? std::string(".") : self.substr(0, slash)) + "/libsplinter_hip.so";
    } else {
      path = "libsplinter_hip.so";
    }
  }
  g_hip_handle = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!g_hip_handle) fprintf(stderr, "libsplinter: cannot load HBM backend %s: %s\n", path.c_str(), dlerror());
  return g_hip_handle;
}

spl::HbmFactory hbm_factory() {
  std::lock_guard<std::mutex> lk(g_hbm_mu);
  if (g_hbm_factory) return g_hbm_factory;
  void* h = hip_handle_locked();
  if (!h) return nullptr;
  g_hbm_factory = (spl::HbmFactory)dlsym(h, "spl_hbm_factory");
  return g_hbm_factory;
}

bool default_embeddings() {
  const char* v = getenv("SPLINTER_EMBEDDINGS");
  return v ? env_true(v) : true;
}

StoreBase* do_create(const char* raw, size_t slots, size_t max_val, unsigned flags, int* err) {
  Parsed p = parse_name(raw);
  bool emb = (flags & SPL_CREATE_EMBEDDINGS) ? true : (flags & SPL_CREATE_NO_EMBEDDINGS) ? false : default_embeddings();
  if (p.kind == Kind::Node) return spl::NodeStore::create(p.name, slots, max_val, emb, err);
  if (p.kind == Kind::Hbm) {
    spl::HbmFactory f = hbm_factory();
    if (!f) { *err = ENOSYS; return nullptr; }
    return f(p.name.c_str(), slots, max_val, emb ? spl::kCreateEmbeddings : spl::kCreateNoEmbeddings, 1, err);
  }
  bool file = p.kind == Kind::File || (flags & SPL_CREATE_PERSISTENT);
  return spl::HostStore::create(p.name.c_str(), file, slots, max_val, emb, err);
}

StoreBase* do_open(const char* raw, int* err) {
  Parsed p = parse_name(raw);
  if (p.kind == Kind::Node) return spl::NodeStore::open(p.name, err);
  if (p.kind == Kind::Hbm) {
    spl::HbmFactory f = hbm_factory();
    if (!f) { *err = ENOSYS; return nullptr; }
    return f(p.name.c_str(), 0, 0, 0, 0, err);
  }
  return spl::HostStore::open(p.name.c_str(), p.kind == Kind::File, err);
}

void replace_current(StoreBase* s) {
  if (g_cur && g_cur != s) delete g_cur;
  g_cur = s;
}

}  // namespace

namespace spl {
HbmFactory load_hbm_factory() { return hbm_factory(); }
void* hbm_symbol(const char* sym) {
  std::lock_guard<std::mutex> lk(g_hbm_mu);
  void* h = hip_handle_locked();
  return h ? dlsym(h, sym) : nullptr;
}
}  // namespace spl

extern "C" {

// ------------------------------------------------------------ lifecycle --
int splinter_create(const char* name, size_t slots, size_t max_val) {
  if (!name) return -2;
  if (slots == 0 || max_val == 0) { errno = ENOTSUP; return -2; }
  int err = 0;
  StoreBase* s = do_create(name, slots, max_val, 0, &err);
  if (!s) { errno = err; return -1; }
  replace_current(s);
  return 0;
}

int splinter_open(const char* name) {
  if (!name) return -2;
  int err = 0;
  StoreBase* s = do_open(name, &err);
  if (!s) { errno = err; return -1; }
  replace_current(s);
  return 0;
}

int splinter_create_or_open(const char* name, size_t slots, size_t max_val) {
  return splinter_create(name, slots, max_val) == 0 ? 0 : splinter_open(name);
}

int splinter_open_or_create(const char* name, size_t slots, size_t max_val) {
  return splinter_open(name) == 0 ? 0 : splinter_create(name, slots, max_val);
}

void* splinter_open_numa(const char* name, int node) {
  // Map the store and bind its pages to `node` (MPOL_BIND=2, MF_STRICT|MF_MOVE).
  if (!name || node < 0 || node >= 64) return nullptr;
  int err = 0;
  spl::HostStore* s = spl::HostStore::open(parse_name(name).name.c_str(), parse_name(name).kind == Kind::File, &err);
  if (!s) { errno = err; return nullptr; }
  unsigned long mask = 1ul << node;
#ifdef SYS_mbind
  if (syscall(SYS_mbind, s->base(), s->total_bytes(), 2 /*MPOL_BIND*/, &mask, 64, (1u << 0) | (1u << 1)) != 0)
    perror("mbind");
#endif
  replace_current(s);
  return s->base();
}

void splinter_close(void) { replace_current(nullptr); }

uint64_t splinter_now_ticks(void) { return spl::now_ticks(); }
uint64_t splinter_now(void) { return spl::now_ticks(); }

// ------------------------------------------------------------- handles --
spl_store* spl_store_create(const char* name, size_t slots, size_t max_val, unsigned flags, int* err) {
  int e = 0;
  StoreBase* s = name ? do_create(name, slots, max_val, flags, &e) : nullptr;
  if (err) *err = s ? 0 : (e ? e : EINVAL);
  return (spl_store*)s;
}
spl_store* spl_store_open(const char* name, int* err) {
  int e = 0;
  StoreBase* s = name ? do_open(name, &e) : nullptr;
  if (err) *err = s ? 0 : (e ? e : EINVAL);
  return (spl_store*)s;
}
void spl_store_close(spl_store* h) {
  StoreBase* s = (StoreBase*)h;
  if (!s) return;
  if (s == g_cur) g_cur = nullptr;
  delete s;
}
int spl_store_use(spl_store* h) { g_cur = (StoreBase*)h; return 0; }
spl_store* spl_store_current(void) { return (spl_store*)g_cur.load(); }
const char* spl_store_backend(spl_store* h) { return h ? ((StoreBase*)h)->backend() : "none"; }
int spl_store_geometry(spl_store* h, uint32_t* slots, uint32_t* max_val, uint32_t* stride) {
  if (!h) return -2;
  spl::Geometry g = ((StoreBase*)h)->geometry();
  if (slots) *slots = g.slots;
  if (max_val) *max_val = g.max_val;
  if (stride) *stride = g.stride;
  return 0;
}
void* spl_store_base(spl_store* h) {
  auto* s = dynamic_cast<spl::HostStore*>((StoreBase*)h);
  return s ? s->base() : nullptr;
}
size_t spl_store_bytes(spl_store* h) {
  auto* s = dynamic_cast<spl::HostStore*>((StoreBase*)h);
  return s ? s->total_bytes() : (h ? ((StoreBase*)h)->geometry().total_bytes() : 0);
}
int spl_store_sync(spl_store* h, int async) {
  // Durability point for file-backed stores (the reference maps MAP_SHARED and
  // never msyncs, SURVEY §5 checkpoint/resume).  shm: nothing to flush.
  auto* s = dynamic_cast<spl::HostStore*>((StoreBase*)h);
  if (!s) { errno = EOPNOTSUPP; return -1; }
  if (!s->base()) { errno = EINVAL; return -1; }
  return msync(s->base(), s->total_bytes(), async ? MS_ASYNC : MS_SYNC);
}
long spl_list_copy(char* buf, size_t cap) {
  // Key names of the current store, NUL-separated, copied out (FFI bindings
  // cannot safely walk splinter_list's pointers into the mapping).  Returns
  // bytes written, or -(bytes needed) when `cap` is too small.
  spl_store* h = spl_store_current();
  if (!h) { errno = ENOTCONN; return 0; }
  uint32_t slots = 0, mv = 0, stride = 0;
  spl_store_geometry(h, &slots, &mv, &stride);
  std::vector<char*> names(slots ? slots : 1);
  size_t n = 0;
  if (((StoreBase*)h)->list(names.data(), names.size(), &n) != 0) return 0;
  size_t need = 0;
  for (size_t i = 0; i < n; ++i) need += strlen(names[i]) + 1;
  if (need > cap) return -(long)need;
  size_t off = 0;
  for (size_t i = 0; i < n; ++i) {
    const size_t L = strlen(names[i]) + 1;
    memcpy(buf + off, names[i], L);
    off += L;
  }
  return (long)off;
}
int spl_unlink(const char* raw) {
  Parsed p = parse_name(raw);
  if (p.kind == Kind::File) return unlink(p.name.c_str());
  if (p.kind == Kind::Hbm) {
    (void)shm_unlink((p.name + ".ring").c_str());  // the ring server's segment (a crashed owner's)
    return shm_unlink((p.name + ".hbm").c_str());
  }
  if (p.kind == Kind::Node) {
    // every shard of the node, then its descriptor.  The shard count and backend come straight from
    // the mapped descriptor (no NodeStore::open, which would import every arena and refuses a node
    // whose create failed half way), so an unusable node can still be cleaned up.
    int rc = 0;
    const std::string dn = p.name + ".node";
    const int fd = shm_open(dn.c_str(), O_RDONLY | O_CLOEXEC, 0);
    if (fd >= 0) {
      struct stat st;
      uint32_t k = 0, backend = 0;
      if (fstat(fd, &st) == 0 && (size_t)st.st_size >= sizeof(spl::NodeDesc)) {
        void* m = mmap(nullptr, sizeof(spl::NodeDesc), PROT_READ, MAP_SHARED, fd, 0);
        if (m != MAP_FAILED) {
          const auto* d = (const spl::NodeDesc*)m;
          k = d->nshards;
          backend = d->backend;
          munmap(m, sizeof(spl::NodeDesc));
        }
      }
      close(fd);
      if (k > (uint32_t)spl::kNodeMaxShards || backend > 1) k = 0;
      for (uint32_t i = 0; i < k; ++i) {
        const std::string sn = spl::node_shard_name(p.name, (int)i, backend);
        if (spl_unlink(sn.c_str()) != 0 && errno != ENOENT) rc = -1;
      }
    }
    if (shm_unlink(dn.c_str()) != 0) rc = -1;
    return rc;
  }
  return shm_unlink(p.name.c_str());
}
const char* spl_version(void) { return "libsplinter_amd 0.1.0 (format v4)"; }
const char* spl_build(void) { return SPL_BUILD_ID; }
long spl_find_slot(spl_store* h, const char* key) {
  auto* s = dynamic_cast<spl::HostStore*>((StoreBase*)h);
  if (!s || !key) return -1;
  return s->find(spl::KeyRef(key));
}
uint64_t spl_hash_key(const char* key) { return spl::KeyRef(key).hash; }

}  // extern "C"

// ------------------------------------------- forwarded operations --------
#define PREPEND_H(...) (spl_store* h, __VA_ARGS__)
#define DUAL(RET, NAME, ERR, CALL, PARAMS)                                  \
  extern "C" RET splinter_##NAME PARAMS {                                   \
    StoreBase* s = g_cur;                                                   \
    if (!s) return ERR;                                                     \
    return s->CALL;                                                         \
  }                                                                         \
  extern "C" RET spl_##NAME PREPEND_H PARAMS {                              \
    StoreBase* s = (StoreBase*)h;                                           \
    if (!s) return ERR;                                                     \
    return s->CALL;                                                         \
  }
#define DUAL0(RET, NAME, ERR, CALL)                                         \
  extern "C" RET splinter_##NAME(void) {                                    \
    StoreBase* s = g_cur;                                                   \
    if (!s) return ERR;                                                     \
    return s->CALL;                                                         \
  }                                                                         \
  extern "C" RET spl_##NAME(spl_store* h) {                                 \
    StoreBase* s = (StoreBase*)h;                                           \
    if (!s) return ERR;                                                     \
    return s->CALL;                                                         \
  }

DUAL(int, set_mop, -2, set_mop(mode), (unsigned int mode))
DUAL0(int, get_mop, -2, get_mop())
DUAL(int, get_header_snapshot, -2, header_snapshot(snap), (splinter_header_snapshot_t* snap))
DUAL(int, set, -2, set(key, val, len), (const char* key, const void* val, size_t len))
DUAL(int, unset, -2, unset(key), (const char* key))
DUAL(int, get, -2, get(key, buf, buf_sz, out_sz), (const char* key, void* buf, size_t buf_sz, size_t* out_sz))
DUAL(int, list, -2, list(out_keys, max_keys, out_count), (char** out_keys, size_t max_keys, size_t* out_count))
DUAL(int, poll, -2, poll(key, timeout_ms), (const char* key, uint64_t timeout_ms))
DUAL(int, get_slot_snapshot, -2, slot_snapshot(key, snap), (const char* key, splinter_slot_snapshot_t* snap))
DUAL(int, append, -2, append(key, data, len, new_len), (const char* key, const void* data, size_t len, size_t* new_len))
DUAL(const void*, get_raw_ptr, nullptr, raw_ptr(key, out_sz, out_epoch), (const char* key, size_t* out_sz, uint64_t* out_epoch))
DUAL(uint64_t, get_epoch, 0, epoch_of(key), (const char* key))
DUAL(int, set_as_system, -2, set_as_system(key), (const char* key))
DUAL(int, set_embedding, -2, set_embedding(key, vec), (const char* key, const float* vec))
DUAL(int, get_embedding, -2, get_embedding(key, out), (const char* key, float* out))
DUAL(int, set_named_type, -2, set_named_type(key, mask), (const char* key, uint16_t mask))
DUAL(int, set_slot_time, -2, set_slot_time(key, mode, epoch, offset), (const char* key, unsigned short mode, uint64_t epoch, size_t offset))
DUAL(int, integer_op, -2, integer_op(key, op, mask), (const char* key, splinter_integer_op_t op, const void* mask))
DUAL(int, bump_slot, -2, bump(key), (const char* key))
DUAL(int, retrain_slot, -2, retrain(key), (const char* key))
DUAL(int, set_label, -2, set_label(key, mask), (const char* key, uint64_t mask))
DUAL(int, unset_label, -2, unset_label(key, mask), (const char* key, uint64_t mask))
DUAL(int, watch_register, -2, watch_register(key, group), (const char* key, uint8_t group))
DUAL(int, watch_unregister, -2, watch_unregister(key, group), (const char* key, uint8_t group))
DUAL(int, watch_label_register, -2, watch_label_register(mask, group), (uint64_t mask, uint8_t group))
DUAL(int, pulse_keygroup, -2, pulse_keygroup(key), (const char* key))
DUAL(uint64_t, get_signal_count, 0, signal_count(group), (uint8_t group))
DUAL0(int, event_bus_init, -1, event_bus_init())
DUAL0(int, event_bus_open, -1, event_bus_open())
DUAL(int, shard_claim_ex, -2, shard_claim_ex(id, pid, intent, prio, dur, at), (uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio, uint64_t dur, uint64_t at))
DUAL(int, shard_rebid, -2, shard_rebid(id, intent, prio, dur), (uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur))
DUAL(int, shard_release, -2, shard_release(id), (uint32_t id))
DUAL(uint32_t, shard_election, 0, shard_election(out_intent), (uint8_t* out_intent))
DUAL(int, shard_table_snapshot, -2, shard_table(out, max), (struct splinter_shard_bid_snapshot* out, size_t max))
DUAL(int, madvise, -2, madvise(id, addr, len, advice, timeout), (uint32_t id, void* addr, size_t len, int advice, uint64_t timeout))

extern "C" {

void splinter_purge(void) { if (g_cur) g_cur.load()->purge(); }
int spl_signal_add(spl_store* h, uint8_t group, uint64_t delta) {
  return h ? ((StoreBase*)h)->signal_add(group, delta) : -2;
}
void spl_purge(spl_store* h) { if (h) ((StoreBase*)h)->purge(); }

int splinter_shard_claim(uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur) {
  if (!g_cur) return -2;
  return g_cur.load()->shard_claim_ex(id, (uint32_t)getpid(), intent, prio, dur, spl::now_ticks());
}
int spl_shard_claim(spl_store* h, uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur) {
  if (!h) return -2;
  return ((StoreBase*)h)->shard_claim_ex(id, (uint32_t)getpid(), intent, prio, dur, spl::now_ticks());
}
int splinter_shard_is_sovereign(uint32_t id) {
  if (!g_cur) return -2;
  return (id != 0 && g_cur.load()->shard_election(nullptr) == id) ? 1 : 0;
}

void splinter_enumerate_matches(uint64_t mask, void (*cb)(const char*, uint64_t, void*), void* ud) {
  if (g_cur) g_cur.load()->enumerate(mask, cb, ud);
}
void spl_enumerate_matches(spl_store* h, uint64_t mask, void (*cb)(const char*, uint64_t, void*), void* ud) {
  if (h) ((StoreBase*)h)->enumerate(mask, cb, ud);
}

void splinter_event_bus_get_dirty(uint64_t* out, size_t words) { if (g_cur) g_cur.load()->event_bus_dirty(out, words); }
void spl_event_bus_get_dirty(spl_store* h, uint64_t* out, size_t words) { if (h) ((StoreBase*)h)->event_bus_dirty(out, words); }

int splinter_event_bus_wait(int fd, uint64_t timeout_ms) {
  if (fd < 0) return -1;
  struct pollfd p = {fd, POLLIN, 0};
  int t = timeout_ms == UINT64_MAX ? -1 : (timeout_ms > 0x7fffffff ? 0x7fffffff : (int)timeout_ms);
  if (::poll(&p, 1, t) <= 0) return -1;
  uint64_t v;
  return read(fd, &v, sizeof(v)) == (ssize_t)sizeof(v) ? 0 : -1;
}
void splinter_event_bus_close(int fd) { if (fd >= 0) close(fd); }

void splinter_pulse_watchers(struct splinter_slot* slot) { if (g_cur && slot) g_cur.load()->pulse_slot(slot); }

// flag helpers operate on the header pointer they are given; NULL means the
// current store (works for the HBM backend, whose header is not host-mapped).
void splinter_config_set(struct splinter_header* hdr, uint8_t mask) {
  if (hdr) __atomic_fetch_or(&hdr->core_flags, mask, __ATOMIC_ACQ_REL);
  else if (g_cur) g_cur.load()->config_or(mask);
}
void splinter_config_clear(struct splinter_header* hdr, uint8_t mask) {
  if (hdr) __atomic_fetch_and(&hdr->core_flags, (uint8_t)~mask, __ATOMIC_ACQ_REL);
  else if (g_cur) g_cur.load()->config_and((uint8_t)~mask);
}
int splinter_config_test(struct splinter_header* hdr, uint8_t mask) {
  uint8_t f = hdr ? __atomic_load_n(&hdr->core_flags, __ATOMIC_ACQUIRE) : (g_cur ? g_cur.load()->config_get() : 0);
  return (f & mask) != 0;
}
uint8_t splinter_config_snapshot(struct splinter_header* hdr) {
  return hdr ? __atomic_load_n(&hdr->core_flags, __ATOMIC_ACQUIRE) : (g_cur ? g_cur.load()->config_get() : 0);
}
void splinter_slot_usr_set(struct splinter_slot* s, uint16_t m) { if (s) __atomic_fetch_or(&s->user_flag, (uint8_t)m, __ATOMIC_ACQ_REL); }
void splinter_slot_usr_clear(struct splinter_slot* s, uint16_t m) { if (s) __atomic_fetch_and(&s->user_flag, (uint8_t)~m, __ATOMIC_ACQ_REL); }
int splinter_slot_usr_test(struct splinter_slot* s, uint16_t m) { return s ? (__atomic_load_n(&s->user_flag, __ATOMIC_ACQUIRE) & m) != 0 : 0; }
uint16_t splinter_slot_usr_snapshot(struct splinter_slot* s) { return s ? __atomic_load_n(&s->user_flag, __ATOMIC_ACQUIRE) : 0; }

// ------------------------------------------------------------- tandem --
static int tandem_set(StoreBase* s, const char* base, const void** vals, const size_t* lens, uint8_t orders) {
  if (!s || !base || !vals || !lens) return -2;
  if (s->set(base, vals[0], lens[0]) != 0) return -1;
  char name[SPLINTER_KEY_MAX];
  for (unsigned i = 1; i < orders; ++i) {
    snprintf(name, sizeof(name), "%s%s%u", base, SPL_ORDER_ACCESSOR, i);
    if (s->set(name, vals[i], lens[i]) != 0) return -1;
  }
  return 0;
}
static void tandem_unset(StoreBase* s, const char* base, uint8_t orders) {
  if (!s || !base) return;
  s->unset(base);
  char name[SPLINTER_KEY_MAX];
  for (unsigned i = 1; i < orders; ++i) {
    snprintf(name, sizeof(name), "%s%s%u", base, SPL_ORDER_ACCESSOR, i);
    s->unset(name);
  }
}
int splinter_client_set_tandem(const char* base, const void** vals, const size_t* lens, uint8_t orders) {
  return tandem_set(g_cur, base, vals, lens, orders);
}
void splinter_client_unset_tandem(const char* base, uint8_t orders) { tandem_unset(g_cur, base, orders); }
int spl_client_set_tandem(spl_store* h, const char* base, const void** vals, const size_t* lens, uint8_t orders) {
  return tandem_set((StoreBase*)h, base, vals, lens, orders);
}
void spl_client_unset_tandem(spl_store* h, const char* base, uint8_t orders) { tandem_unset((StoreBase*)h, base, orders); }

}  // extern "C"
