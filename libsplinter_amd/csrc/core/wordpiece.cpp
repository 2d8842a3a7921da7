// wordpiece.cpp — BERT WordPiece tokenizer for the embedding daemon (K10 of
// SURVEY §2.10).  The reference delegates tokenisation to llama.cpp
// (/root/reference/splinference.cpp:210-217); here it is native C++ driven
// by the vocabulary stored in the GGUF (tokenizer.ggml.tokens).
//
// Two vocabulary conventions are accepted and detected automatically:
//   * llama.cpp / GGUF ("WPM"): word-initial pieces carry U+2581 "▁",
//     continuation pieces are bare;
//   * HF BERT: word-initial pieces are bare, continuations carry "##".
// Pre-tokenisation follows BERT's basic tokenizer: clean control chars,
// lowercase, strip common Latin accents, split on whitespace, punctuation and
// CJK ideographs; then greedy longest-match-first WordPiece per word, a word
// with no decomposition (or longer than 100 code points) becomes [UNK].
// Batch encoding fans out over a small thread pool.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <unistd.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

namespace {

// Open-addressing piece table keyed by byte strings, looked up with string_views straight into the
// normalised text (no candidate string is built per lookup).  First insertion of a key wins, as
// std::unordered_map::emplace did.
struct PieceTable {
  struct Entry { uint64_t h; uint32_t off, len; int32_t id; };
  std::vector<Entry> slots;  // id < 0: empty
  std::string pool;
  uint64_t mask = 0;

  static uint64_t hash(const char* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ (unsigned char)p[i]) * 1099511628211ull;
    return h ^ (h >> 29);
  }
  void init(size_t n) {
    size_t cap = 16;
    while (cap < n * 2 + 16) cap <<= 1;
    slots.assign(cap, Entry{0, 0, 0, -1});
    mask = cap - 1;
  }
  void insert(std::string_view k, int32_t id) {
    const uint64_t h = hash(k.data(), k.size());
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      Entry& e = slots[i];
      if (e.id < 0) {
        e = Entry{h, (uint32_t)pool.size(), (uint32_t)k.size(), id};
        pool.append(k.data(), k.size());
        return;
      }
      if (e.h == h && e.len == k.size() && std::memcmp(pool.data() + e.off, k.data(), k.size()) == 0) return;
    }
  }
  int32_t find(const char* p, size_t n) const {
    const uint64_t h = hash(p, n);
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      const Entry& e = slots[i];
      if (e.id < 0) return -1;
      if (e.h == h && e.len == n && std::memcmp(pool.data() + e.off, p, n) == 0) return e.id;
    }
  }
};

struct Tok {
  // word-initial lookups (WPM: "▁" + piece, stored stripped; BERT: the bare piece) and continuation
  // lookups (WPM: the bare piece; BERT: "##" + piece, stored stripped) -- the exact candidates the
  // greedy longest-match builds
  PieceTable first, cont;
  int32_t cls = -1, sep = -1, unk = 0;
  bool wpm = false;          // "▁" convention
  size_t max_piece = 1;      // longest vocab entry in bytes
};

// ---------------------------------------------------------- UTF-8 utils --
inline uint32_t decode(const unsigned char* s, size_t n, size_t& i) {
  const unsigned char c = s[i];
  if (c < 0x80) { i += 1; return c; }
  if ((c >> 5) == 6 && i + 1 < n) { uint32_t r = ((c & 31u) << 6) | (s[i + 1] & 63u); i += 2; return r; }
  if ((c >> 4) == 14 && i + 2 < n) {
    uint32_t r = ((c & 15u) << 12) | ((s[i + 1] & 63u) << 6) | (s[i + 2] & 63u);
    i += 3;
    return r;
  }
  if ((c >> 3) == 30 && i + 3 < n) {
    uint32_t r = ((c & 7u) << 18) | ((s[i + 1] & 63u) << 12) | ((s[i + 2] & 63u) << 6) | (s[i + 3] & 63u);
    i += 4;
    return r;
  }
  i += 1;
  return 0xFFFD;
}

inline void encode(uint32_t cp, std::string& out) {
  if (cp < 0x80) out.push_back((char)cp);
  else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 63))); }
  else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 63)));
    out.push_back((char)(0x80 | (cp & 63)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 63)));
    out.push_back((char)(0x80 | ((cp >> 6) & 63)));
    out.push_back((char)(0x80 | (cp & 63)));
  }
}

inline bool is_space(uint32_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0xA0 || c == 0x3000 || (c >= 0x2000 && c <= 0x200A) ||
         c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F;
}
inline bool is_control(uint32_t c) { return (c < 32 && !is_space(c)) || c == 127 || (c >= 0x80 && c < 0xA0) || c == 0xFFFD; }
inline bool is_punct(uint32_t c) {
  if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126)) return true;
  return (c >= 0x2010 && c <= 0x2027) || (c >= 0x2030 && c <= 0x205E) || (c >= 0x3001 && c <= 0x303F) ||
         (c >= 0xFF01 && c <= 0xFF0F) || c == 0xA1 || c == 0xA7 || c == 0xAB || c == 0xB6 || c == 0xB7 || c == 0xBB ||
         c == 0xBF;
}
inline bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) || (c >= 0x20000 && c <= 0x2A6DF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}

// lowercase + accent folding for the Latin-1 / Latin Extended-A range, Greek and
// Cyrillic capitals (approximation of NFD + Mn stripping used by BERT-uncased)
inline uint32_t fold(uint32_t c) {
  if (c >= 'A' && c <= 'Z') return c + 32;
  if (c < 0xC0) return c;
  static const char* lat = "aaaaaaaceeeeiiiidnooooo*ouuuuyts" "aaaaaaaceeeeiiiidnooooo/ouuuuyty";
  if (c >= 0xC0 && c <= 0xFF) {
    const char m = lat[c - 0xC0];
    if (m == '*' || m == '/') return c == 0xD7 ? 0xD7 : 0xF7;
    if (c == 0xC6 || c == 0xE6) return 0xE6;  // ae ligature kept
    if (c == 0xDF) return 0xDF;               // sharp s
    if (c == 0xDE || c == 0xFE) return 0xFE;  // thorn
    if (c == 0xD0 || c == 0xF0) return 0xF0;  // eth
    return (uint32_t)(unsigned char)m;
  }
  if (c >= 0x100 && c <= 0x17F) {  // Latin Extended-A: strip to base letter
    static const char* ext = "aaaaaaccccccccddddeeeeeeeeeegggggggghhhhiiiiiiiiiiijjjjkkklllllllllllnnnnnnnnnoooooooo"
                             "oorrrrrrsssssssstttttttuuuuuuuuuuuuwwyyyzzzzzzs";
    const size_t k = c - 0x100;
    if (k < strlen(ext)) return (uint32_t)(unsigned char)ext[k];
    return c;
  }
  if (c >= 0x391 && c <= 0x3A9) return c + 32;   // Greek capitals
  if (c >= 0x410 && c <= 0x42F) return c + 32;   // Cyrillic capitals
  if (c >= 0x400 && c <= 0x40F) return c + 80;
  if (c >= 0x300 && c <= 0x36F) return 0;        // combining marks: drop
  return c;
}

// normalised text (folded, control chars dropped) + word spans: whitespace separates words,
// punctuation and CJK ideographs are words of their own
struct Scratch {
  std::string norm;
  std::vector<std::pair<uint32_t, uint32_t>> words;  // (offset, bytes) into norm
  std::vector<uint32_t> cps;
};

void split_words(const char* text, size_t n, Scratch& sc) {
  const unsigned char* s = (const unsigned char*)text;
  sc.norm.clear();
  sc.words.clear();
  size_t start = 0;
  auto flush = [&] {
    if (sc.norm.size() > start) sc.words.emplace_back((uint32_t)start, (uint32_t)(sc.norm.size() - start));
    start = sc.norm.size();
  };
  for (size_t i = 0; i < n;) {
    uint32_t c = decode(s, n, i);
    if (c == 0 || is_control(c)) continue;
    if (is_space(c)) { flush(); continue; }
    c = fold(c);
    if (c == 0) continue;
    if (is_punct(c) || is_cjk(c)) {
      flush();
      encode(c, sc.norm);
      flush();
      continue;
    }
    encode(c, sc.norm);
  }
  flush();
}

void wordpiece(const Tok& t, const char* w, size_t wn, std::vector<uint32_t>& cps, std::vector<int32_t>& out) {
  // code-point boundaries
  cps.clear();
  const unsigned char* s = (const unsigned char*)w;
  for (size_t i = 0; i < wn;) { cps.push_back((uint32_t)i); decode(s, wn, i); }
  if (cps.size() > 100) { out.push_back(t.unk); return; }
  cps.push_back((uint32_t)wn);
  const size_t start_n = out.size();
  const size_t prefix = t.wpm ? 3 : 2;  // bytes of "▁" / "##" counted in a candidate's length
  size_t b = 0;  // index into cps
  while (b + 1 < cps.size()) {
    int32_t found = -1;
    size_t e = cps.size() - 1;
    const PieceTable& tab = b == 0 ? t.first : t.cont;
    const size_t extra = (t.wpm ? b == 0 : b != 0) ? prefix : 0;
    for (; e > b; --e) {
      const size_t bytes = cps[e] - cps[b];
      if (bytes + extra > t.max_piece) continue;
      found = tab.find(w + cps[b], bytes);
      if (found >= 0) break;
    }
    if (found < 0) { out.resize(start_n); out.push_back(t.unk); return; }
    out.push_back(found);
    b = e;
  }
}

int encode_one(const Tok& t, const char* text, size_t n, std::vector<int32_t>& ids, int add_special) {
  thread_local Scratch sc;
  ids.clear();
  if (add_special && t.cls >= 0) ids.push_back(t.cls);
  split_words(text, n, sc);
  for (auto& [off, len] : sc.words) wordpiece(t, sc.norm.data() + off, len, sc.cps, ids);
  if (add_special && t.sep >= 0) ids.push_back(t.sep);
  return (int)ids.size();
}

// Persistent worker pool for batch encoding: spawning a thread per worker per batch cost ~0.5 ms of
// a ~2 ms batch.  Workers are detached and sleep on a condition variable between batches; a batch
// runs on the caller plus up to n-1 workers that claim a slot; the caller returns once every
// claimed slot has finished, and closes the remaining slots so a late waker never runs a stale
// job.  A forked child (different pid) starts a fresh pool.
struct Pool {
  std::mutex mu, run_mu;
  std::condition_variable cv, done;
  std::function<void()> job;
  uint64_t gen = 0;
  int slots = 0, active = 0, nthreads = 0;
  pid_t pid = 0;

  void worker(uint64_t seen) {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return gen != seen; });
      seen = gen;
      if (slots <= 0) continue;
      --slots;
      ++active;
      std::function<void()> j = job;
      lk.unlock();
      j();
      lk.lock();
      if (--active == 0) done.notify_all();
    }
  }

  void run(int n, const std::function<void()>& fn) {
    std::lock_guard<std::mutex> serial(run_mu);
    {
      std::lock_guard<std::mutex> lk(mu);
      if (pid != getpid()) { pid = getpid(); nthreads = 0; }
      while (nthreads < n - 1) {
        std::thread([this, g = gen] { worker(g); }).detach();
        ++nthreads;
      }
      job = fn;
      slots = n - 1;
      ++gen;
    }
    cv.notify_all();
    fn();
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [&] { return active == 0; });
    slots = 0;
    job = nullptr;
  }
};

Pool& pool() {
  static Pool* p = new Pool();  // never destroyed: detached workers may outlive static destructors
  return *p;
}

}  // namespace

extern "C" {

void* spl_tok_create(const char* const* tokens, int n, int cls_id, int sep_id, int unk_id) {
  auto* t = new Tok();
  for (int i = 0; i < n; ++i) {
    const std::string_view s(tokens[i]);
    if (s.size() > t->max_piece) t->max_piece = s.size();
    if (s.substr(0, 3) == "\xE2\x96\x81") t->wpm = true;
  }
  t->first.init((size_t)n);
  t->cont.init((size_t)n);
  for (int i = 0; i < n; ++i) {
    const std::string_view s(tokens[i]);
    if (t->wpm) {
      if (s.substr(0, 3) == "\xE2\x96\x81") t->first.insert(s.substr(3), i);  // "▁" + piece
      t->cont.insert(s, i);                                                    // bare piece
    } else {
      t->first.insert(s, i);                                                   // bare piece
      if (s.substr(0, 2) == "##") t->cont.insert(s.substr(2), i);              // "##" + piece
    }
  }
  t->cls = cls_id;
  t->sep = sep_id;
  t->unk = unk_id >= 0 ? unk_id : 0;
  return t;
}

void spl_tok_free(void* t) { delete (Tok*)t; }

int spl_tok_is_wpm(void* t) { return ((Tok*)t)->wpm ? 1 : 0; }

// Encode one text; writes up to max_out ids, returns the full count.
int spl_tok_encode(void* tp, const char* text, size_t len, int32_t* out, int max_out, int add_special) {
  std::vector<int32_t> ids;
  const int n = encode_one(*(Tok*)tp, text, len, ids, add_special);
  const int m = std::min(n, max_out);
  if (out && m > 0) std::memcpy(out, ids.data(), (size_t)m * 4);
  return n;
}

// Encode a batch.  Sequences are truncated to max_per_seq ids (the full
// length is reported in full_lens so callers can apply the reference's
// context-exceeded policy).  Output is packed: offsets[n+1] into out_flat.
// Returns the total number of ids written, or -1 if out_flat is too small.
int spl_tok_encode_batch(void* tp, const char* const* texts, const size_t* lens, int n, int32_t* out_flat,
                         long cap, int64_t* offsets, int32_t* full_lens, int max_per_seq, int add_special,
                         int threads) {
  const Tok& t = *(Tok*)tp;
  std::vector<std::vector<int32_t>> res((size_t)n);
  std::atomic<int> next{0};
  auto work = [&] {
    for (int i; (i = next.fetch_add(1)) < n;) {
      encode_one(t, texts[i], lens[i], res[(size_t)i], add_special);
    }
  };
  if (threads < 1) threads = 1;
  threads = std::min(threads, std::max(1, n / 8));
  static const bool use_pool = [] {  // SPL_TOK_POOL=0: a thread per worker per batch (A/B)
    const char* e = getenv("SPL_TOK_POOL");
    return !(e && *e == '0');
  }();
  if (threads == 1) {
    work();
  } else if (use_pool) {
    pool().run(threads, work);
  } else {
    std::vector<std::thread> ths;
    for (int k = 1; k < threads; ++k) ths.emplace_back(work);
    work();
    for (auto& th : ths) th.join();
  }
  long pos = 0;
  offsets[0] = 0;
  for (int i = 0; i < n; ++i) {
    auto& v = res[(size_t)i];
    if (full_lens) full_lens[i] = (int32_t)v.size();
    int m = (int)v.size();
    if (m > max_per_seq) {
      m = max_per_seq;
      if (add_special && t.sep >= 0) v[(size_t)m - 1] = t.sep;  // keep the trailing [SEP]
    }
    if (pos + m > cap) return -1;
    std::memcpy(out_flat + pos, v.data(), (size_t)m * 4);
    pos += m;
    offsets[i + 1] = pos;
  }
  return (int)pos;
}

}  // extern "C"
