// fa_wire.cpp — host side of the wire codec (include/flearn_amd.h, "wire codec").
//
// flearn's HTTP mode ships every upload and every global model as base64(pickle.dumps(obj))
// (flearn/common/Encrypt.py:17-44; decoded per upload in Server.ensemble, Server.py:126-131).
// The reference decodes with base64.b64decode + pickle.loads on one core and then the numpy
// arrays are copied again into the aggregation input.  Here:
//   * base64 is decoded / encoded by a persistent thread pool, in 3-byte-aligned pieces;
//   * a restricted pickle scanner walks the opcode stream THROUGH the base64 text (decoding only
//     the small header pieces it needs) and reports each array payload as a (decoded offset,
//     length) pair instead of decoding it; the caller then decodes every payload once, straight
//     into its slot in pinned staging (fa_b64_decode_ranges) — the layout the H2D copy reads.
// Pure host C++: no HIP calls.  The scanner accepts only the opcodes and globals that pickled
// dicts / lists / tuples of numpy arrays and scalars use; anything else is reported as
// FA_ERR_UNSUPPORTED and the caller falls back to a restricted Python unpickler.
#include <immintrin.h>
#include <algorithm>
#include <pthread.h>

#include <atomic>
#include <cctype>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "flearn_amd.h"

namespace {

thread_local std::string g_wire_error;

int wfail(int code, const char* what) {
  g_wire_error = what;
  return code;
}

// ---------------------------------------------------------------------------------------------
// persistent thread pool: run(n, threads, fn) calls fn(0..n-1) on up to `threads` threads
// (the caller included) and returns when all calls have finished.
// ---------------------------------------------------------------------------------------------
class Pool {
 public:
  void run(int64_t n, int threads, const std::function<void(int64_t)>& fn) {
    if (n <= 0) return;
    if (threads <= 1 || n == 1) {
      for (int64_t i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> serial(run_m_);  // one job at a time
    start(threads - 1);
    Job j;
    j.fn = &fn;
    j.n = n;
    j.seats = threads - 1;
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &j;
      ++gen_;
    }
    cv_.notify_all();
    work(&j);
    {
      std::unique_lock<std::mutex> lk(m_);
      job_ = nullptr;  // no worker can join from now on
      done_cv_.wait(lk, [&] { return j.active == 0; });
    }
  }

  static Pool& get() {
    static Pool* p = [] {
      pthread_atfork(nullptr, nullptr, [] { g_forked = true; });
      return new Pool();
    }();
    if (g_forked) {  // a forked child has no workers: start a fresh pool (the old one leaks)
      g_forked = false;
      p = new Pool();
    }
    return *p;
  }

 private:
  struct Job {
    const std::function<void(int64_t)>* fn = nullptr;
    int64_t n = 0;
    std::atomic<int64_t> next{0};
    int seats = 0;   // workers that may still join (guarded by m_)
    int active = 0;  // workers inside work() (guarded by m_)
  };

  static inline bool g_forked = false;

  void start(int want) {
    const int hw = (int)std::thread::hardware_concurrency();
    const int cap = (hw > 1 ? hw - 1 : 1) < 63 ? (hw > 1 ? hw - 1 : 1) : 63;
    if (want > cap) want = cap;
    while ((int)ws_.size() < want) ws_.emplace_back([this] { loop(); });
  }

  static void work(Job* j) {
    for (int64_t i = j->next.fetch_add(1); i < j->n; i = j->next.fetch_add(1)) (*j->fn)(i);
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      Job* j = nullptr;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (!job_ || job_->seats <= 0) continue;
        j = job_;
        --j->seats;
        ++j->active;
      }
      work(j);
      {
        std::lock_guard<std::mutex> lk(m_);
        if (--j->active == 0) done_cv_.notify_all();
      }
    }
  }

  std::vector<std::thread> ws_;
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_cv_;
  Job* job_ = nullptr;
  uint64_t gen_ = 0;
};

int clamp_threads(int32_t t) {
  if (t > 0) return t;
  const int hw = (int)std::thread::hardware_concurrency();
  return hw < 1 ? 1 : (hw > 16 ? 16 : hw);
}

// ---------------------------------------------------------------------------------------------
// base64 (RFC 4648 alphabet, '=' padding) — what base64.b64encode emits
// ---------------------------------------------------------------------------------------------
constexpr char kAlpha[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
constexpr uint32_t kBad = 0x01000000u;

struct Tables {
  uint32_t d0[256], d1[256], d2[256], d3[256];
  uint16_t e2[4096];  // 12 bits -> two output chars (little-endian pair)
  Tables() {
    for (int c = 0; c < 256; ++c) d0[c] = d1[c] = d2[c] = d3[c] = kBad;
    for (uint32_t v = 0; v < 64; ++v) {
      const uint8_t c = (uint8_t)kAlpha[v];
      d0[c] = v << 18;
      d1[c] = v << 12;
      d2[c] = v << 6;
      d3[c] = v;
    }
    for (int v = 0; v < 4096; ++v)
      e2[v] = (uint16_t)((uint8_t)kAlpha[v >> 6] | ((uint16_t)(uint8_t)kAlpha[v & 63] << 8));
  }
};
const Tables& T() {
  static const Tables t;
  return t;
}

// AVX2 decode of 8 groups (32 characters -> 24 bytes) per step: validation and translation by
// nibble lookups (vpshufb), bit packing by vpmaddubsw / vpmaddwd, then a byte shuffle and a lane
// permute (the published Mula-Lemire scheme).  Runs while >= 11 groups remain, so the 32-byte
// store (24 decoded bytes + 8 that later groups overwrite) stays inside this call's output.
// Returns the groups decoded; stops early at a block holding a non-alphabet character, which the
// scalar loop then reports.
__attribute__((target("avx2"))) int64_t dec_groups_avx2(const uint8_t* s, int64_t ng, uint8_t* d) {
  const __m256i lut_lo = _mm256_setr_epi8(0x15, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x13, 0x1A,
                                          0x1B, 0x1B, 0x1B, 0x1A, 0x15, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11,
                                          0x11, 0x11, 0x13, 0x1A, 0x1B, 0x1B, 0x1B, 0x1A);
  const __m256i lut_hi = _mm256_setr_epi8(0x10, 0x10, 0x01, 0x02, 0x04, 0x08, 0x04, 0x08, 0x10, 0x10, 0x10, 0x10,
                                          0x10, 0x10, 0x10, 0x10, 0x10, 0x10, 0x01, 0x02, 0x04, 0x08, 0x04, 0x08,
                                          0x10, 0x10, 0x10, 0x10, 0x10, 0x10, 0x10, 0x10);
  const __m256i lut_roll = _mm256_setr_epi8(0, 16, 19, 4, -65, -65, -71, -71, 0, 0, 0, 0, 0, 0, 0, 0, 0, 16, 19, 4,
                                            -65, -65, -71, -71, 0, 0, 0, 0, 0, 0, 0, 0);
  const __m256i mask_2f = _mm256_set1_epi8(0x2F);
  const __m256i pack_ab = _mm256_set1_epi32(0x01400140);
  const __m256i pack_abc = _mm256_set1_epi32(0x00011000);
  const __m256i shuf = _mm256_setr_epi8(2, 1, 0, 6, 5, 4, 10, 9, 8, 14, 13, 12, -1, -1, -1, -1, 2, 1, 0, 6, 5, 4, 10,
                                        9, 8, 14, 13, 12, -1, -1, -1, -1);
  const __m256i perm = _mm256_setr_epi32(0, 1, 2, 4, 5, 6, 7, 7);
  int64_t g = 0;
  for (; g + 11 <= ng; g += 8) {
    __m256i str = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 4 * g));
    const __m256i hi_nib = _mm256_and_si256(_mm256_srli_epi32(str, 4), mask_2f);
    const __m256i lo_nib = _mm256_and_si256(str, mask_2f);
    const __m256i hi = _mm256_shuffle_epi8(lut_hi, hi_nib);
    const __m256i lo = _mm256_shuffle_epi8(lut_lo, lo_nib);
    if (!_mm256_testz_si256(lo, hi)) break;
    const __m256i eq_2f = _mm256_cmpeq_epi8(str, mask_2f);
    str = _mm256_add_epi8(str, _mm256_shuffle_epi8(lut_roll, _mm256_add_epi8(eq_2f, hi_nib)));
    __m256i out = _mm256_madd_epi16(_mm256_maddubs_epi16(str, pack_ab), pack_abc);
    out = _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(out, shuf), perm);
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(d + 3 * g), out);
  }
  return g;
}

const bool kAvx2 = __builtin_cpu_supports("avx2");

// Decode `ng` full (unpadded) groups; returns false on a non-alphabet character.
inline bool dec_groups(const uint8_t* s, int64_t ng, uint8_t* d) {
  const Tables& t = T();
  uint32_t bad = 0;
  int64_t g = 0;
  if (kAvx2 && ng >= 11) {
    const int64_t done = dec_groups_avx2(s, ng, d);
    s += 4 * done, d += 3 * done, ng -= done;
  }
  for (; g + 4 <= ng; g += 4, s += 16, d += 12) {
#pragma GCC unroll 4
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = t.d0[s[4 * k]] | t.d1[s[4 * k + 1]] | t.d2[s[4 * k + 2]] | t.d3[s[4 * k + 3]];
      bad |= x;
      d[3 * k] = (uint8_t)(x >> 16);
      d[3 * k + 1] = (uint8_t)(x >> 8);
      d[3 * k + 2] = (uint8_t)x;
    }
  }
  for (; g < ng; ++g, s += 4, d += 3) {
    const uint32_t x = t.d0[s[0]] | t.d1[s[1]] | t.d2[s[2]] | t.d3[s[3]];
    bad |= x;
    d[0] = (uint8_t)(x >> 16);
    d[1] = (uint8_t)(x >> 8);
    d[2] = (uint8_t)x;
  }
  return (bad & 0xFF000000u) == 0;
}

// One group that may carry padding ("xx==" -> 1 byte, "xxx=" -> 2); returns bytes or -1.
inline int dec_last(const uint8_t* s, uint8_t* d) {
  const Tables& t = T();
  if (s[2] == '=' && s[3] == '=') {
    const uint32_t x = t.d0[s[0]] | t.d1[s[1]];
    if (x & 0xFF000000u) return -1;
    d[0] = (uint8_t)(x >> 16);
    return 1;
  }
  if (s[3] == '=') {
    const uint32_t x = t.d0[s[0]] | t.d1[s[1]] | t.d2[s[2]];
    if (x & 0xFF000000u) return -1;
    d[0] = (uint8_t)(x >> 16);
    d[1] = (uint8_t)(x >> 8);
    return 2;
  }
  return dec_groups(s, 1, d) ? 3 : -1;
}

struct B64 {
  const uint8_t* s;
  int64_t n;       // characters (multiple of 4)
  int64_t ng;      // groups
  int pad;         // '=' in the last group
  int64_t total;   // decoded bytes
  bool ok;
  B64(const char* src, int64_t len) : s((const uint8_t*)src), n(len), ng(0), pad(0), total(0), ok(false) {
    if (len < 0 || (len & 3) || (len && !src)) return;
    ng = len / 4;
    if (len) {
      pad = (s[len - 1] == '=') + (s[len - 2] == '=');
      if (pad == 1 && s[len - 2] == '=') return;
    }
    total = ng * 3 - pad;
    ok = true;
  }
  int64_t full_groups() const { return pad ? ng - 1 : ng; }
  // decode group g into tmp; returns its byte count or -1
  int group(int64_t g, uint8_t* tmp) const {
    if (g == ng - 1 && pad) return dec_last(s + 4 * g, tmp);
    return dec_groups(s + 4 * g, 1, tmp) ? 3 : -1;
  }
  // decoded bytes [o, o+len) -> dst
  bool range(int64_t o, int64_t len, uint8_t* dst) const {
    if (o < 0 || len < 0 || o + len > total) return false;
    uint8_t tmp[3];
    while (len > 0 && (o % 3 != 0)) {  // head: partial group
      const int c = group(o / 3, tmp);
      if (c < 0) return false;
      int k = (int)(o % 3);
      int64_t take = c - k < len ? c - k : len;
      std::memcpy(dst, tmp + k, (size_t)take);
      dst += take, o += take, len -= take;
    }
    int64_t g = o / 3, nfull = len / 3;
    const int64_t lim = full_groups() - g;
    if (nfull > lim) nfull = lim > 0 ? lim : 0;
    if (nfull > 0) {
      if (!dec_groups(s + 4 * g, nfull, dst)) return false;
      dst += 3 * nfull, o += 3 * nfull, len -= 3 * nfull;
    }
    if (len > 0) {  // tail: partial or padded group
      const int c = group(o / 3, tmp);
      if (c < 0 || c < len) return false;
      std::memcpy(dst, tmp, (size_t)len);
    }
    return true;
  }
};

constexpr int64_t kPiece = 3 * 87382;  // ~256 KiB decoded per task

void enc_groups(const uint8_t* s, int64_t ng, char* d) {
  const Tables& t = T();
  for (int64_t g = 0; g < ng; ++g, s += 3, d += 4) {
    const uint32_t v = ((uint32_t)s[0] << 16) | ((uint32_t)s[1] << 8) | s[2];
    const uint16_t a = t.e2[v >> 12], b = t.e2[v & 4095];
    std::memcpy(d, &a, 2);
    std::memcpy(d + 2, &b, 2);
  }
}

// ---------------------------------------------------------------------------------------------
// restricted pickle scanner
// ---------------------------------------------------------------------------------------------
struct MemReader {  // decoded bytes in memory
  const uint8_t* p;
  int64_t n, pos = 0;
  bool read(int64_t len, uint8_t* out) {
    if (len < 0 || pos + len > n) return false;
    std::memcpy(out, p + pos, (size_t)len);
    pos += len;
    return true;
  }
  bool skip(int64_t len) {
    if (len < 0 || pos + len > n) return false;
    pos += len;
    return true;
  }
};

struct B64Reader {  // decodes the base64 text on demand, through a small window
  const B64& b;
  int64_t pos = 0;
  std::vector<uint8_t> win;
  int64_t w0 = 0, w1 = 0;  // window covers decoded [w0, w1)
  // 4 KiB: the scanner reads headers (a few hundred bytes between payloads it skips); a wider
  // window would decode payload bytes that fa_b64_decode_ranges decodes again
  explicit B64Reader(const B64& bb) : b(bb) { win.resize(1 << 12); }
  bool read(int64_t len, uint8_t* out) {
    if (len < 0 || pos + len > b.total) return false;
    if (pos >= w0 && pos + len <= w1) {
      std::memcpy(out, win.data() + (pos - w0), (size_t)len);
      pos += len;
      return true;
    }
    if (len > (int64_t)win.size() / 2) {  // big read: decode straight
      if (!b.range(pos, len, out)) return false;
      pos += len;
      return true;
    }
    int64_t a = pos - pos % 3, e = a + (int64_t)win.size();
    if (e > b.total) e = b.total;
    if (!b.range(a, e - a, win.data())) return false;
    w0 = a, w1 = e;
    std::memcpy(out, win.data() + (pos - w0), (size_t)len);
    pos += len;
    return true;
  }
  bool skip(int64_t len) {
    if (len < 0 || pos + len > b.total) return false;
    pos += len;
    return true;
  }
};

enum NT : uint8_t { N_NONE, N_BOOL, N_INT, N_FLOAT, N_STR, N_BYTES, N_TUPLE, N_LIST, N_DICT, N_GLOBAL, N_REDUCE };

struct Node {
  NT t = N_NONE;
  bool b = false;
  bool ordered = false;
  int64_t i = 0;
  double f = 0;
  std::string s, s2;  // STR text / small BYTES content; GLOBAL module, name
  int64_t off = 0, len = 0;
  std::vector<int32_t> kids;  // TUPLE/LIST items; DICT k,v,k,v...; REDUCE callable,args
  int32_t state = -1;         // BUILD state
};

constexpr int64_t kSmallBytes = 64;            // BYTES up to this size are decoded (pattern checks)
constexpr size_t kMaxManifest = size_t(1) << 26;  // shared sub-objects could blow the JSON up

struct Scanner {
  std::vector<Node> nodes;
  std::vector<int32_t> stack;
  std::vector<size_t> marks;
  std::unordered_map<int64_t, int32_t> memo;
  int err = FA_OK;
  std::string why;

  int fail(int code, const std::string& w) {
    if (err == FA_OK) {
      err = code;
      why = w;
    }
    return code;
  }
  int32_t add(Node&& n) {
    nodes.push_back(std::move(n));
    return (int32_t)nodes.size() - 1;
  }
  bool pop(int32_t* v) {
    if (stack.empty() || (!marks.empty() && stack.size() <= marks.back())) return false;
    *v = stack.back();
    stack.pop_back();
    return true;
  }
  bool pop_mark(std::vector<int32_t>* items) {
    if (marks.empty()) return false;
    const size_t m = marks.back();
    marks.pop_back();
    items->assign(stack.begin() + (long)m, stack.end());
    stack.resize(m);
    return true;
  }
  static bool allowed_global(const std::string& mod, const std::string& name) {
    const bool mA = mod == "numpy._core.multiarray" || mod == "numpy.core.multiarray";
    const bool mN = mod == "numpy._core.numeric" || mod == "numpy.core.numeric";
    return (mA && (name == "_reconstruct" || name == "scalar")) || (mN && name == "_frombuffer") ||
           (mod == "numpy" && (name == "ndarray" || name == "dtype")) ||
           (mod == "collections" && name == "OrderedDict");
  }

  template <class R>
  int run(R& r) {
    uint8_t op;
    uint8_t buf[8];
    auto rd_u = [&](int nb, uint64_t* v) -> bool {
      if (!r.read(nb, buf)) return false;
      uint64_t x = 0;
      for (int k = nb - 1; k >= 0; --k) x = (x << 8) | buf[k];
      *v = x;
      return true;
    };
    auto push_str = [&](int64_t len) -> bool {
      if (len < 0 || len > (1 << 26)) return false;
      Node n;
      n.t = N_STR;
      n.s.resize((size_t)len);
      if (len && !r.read(len, (uint8_t*)&n.s[0])) return false;
      stack.push_back(add(std::move(n)));
      return true;
    };
    auto push_bytes = [&](int64_t len) -> bool {
      if (len < 0) return false;
      Node n;
      n.t = N_BYTES;
      n.off = r.pos;
      n.len = len;
      if (len <= kSmallBytes) {
        n.s.resize((size_t)len);
        if (len && !r.read(len, (uint8_t*)&n.s[0])) return false;
      } else if (!r.skip(len)) {
        return false;
      }
      stack.push_back(add(std::move(n)));
      return true;
    };
    auto push_int = [&](int64_t v) {
      Node n;
      n.t = N_INT;
      n.i = v;
      stack.push_back(add(std::move(n)));
    };
    auto tuple_of = [&](std::vector<int32_t>&& items) {
      Node n;
      n.t = N_TUPLE;
      n.kids = std::move(items);
      stack.push_back(add(std::move(n)));
    };
    const int64_t kMaxOps = 1ll << 28;
    for (int64_t steps = 0; steps < kMaxOps; ++steps) {
      if (!r.read(1, &op)) return fail(FA_ERR_DATA, "truncated pickle");
      uint64_t u = 0;
      int32_t a = 0, b = 0, c = 0;
      switch (op) {
        case 0x80:  // PROTO
          if (!r.read(1, buf)) return fail(FA_ERR_DATA, "truncated PROTO");
          if (buf[0] < 2 || buf[0] > 5) return fail(FA_ERR_UNSUPPORTED, "pickle protocol < 2");
          break;
        case 0x95:  // FRAME
          if (!rd_u(8, &u)) return fail(FA_ERR_DATA, "truncated FRAME");
          break;
        case '.':  // STOP
          if (stack.size() != 1 || !marks.empty()) return fail(FA_ERR_DATA, "bad stack at STOP");
          return FA_OK;
        case 'N': {
          stack.push_back(add(Node()));
          break;
        }
        case 0x88:
        case 0x89: {
          Node n;
          n.t = N_BOOL;
          n.b = op == 0x88;
          stack.push_back(add(std::move(n)));
          break;
        }
        case 'J':
          if (!rd_u(4, &u)) return fail(FA_ERR_DATA, "truncated BININT");
          push_int((int64_t)(int32_t)(uint32_t)u);
          break;
        case 'K':
          if (!rd_u(1, &u)) return fail(FA_ERR_DATA, "truncated BININT1");
          push_int((int64_t)u);
          break;
        case 'M':
          if (!rd_u(2, &u)) return fail(FA_ERR_DATA, "truncated BININT2");
          push_int((int64_t)u);
          break;
        case 0x8a: {  // LONG1
          if (!rd_u(1, &u)) return fail(FA_ERR_DATA, "truncated LONG1");
          const int nb = (int)u;
          if (nb > 8) return fail(FA_ERR_UNSUPPORTED, "integer wider than 64 bits");
          uint64_t x = 0;
          if (nb && !rd_u(nb, &x)) return fail(FA_ERR_DATA, "truncated LONG1");
          if (nb && nb < 8 && (x >> (8 * nb - 1)) & 1) x |= ~0ull << (8 * nb);  // sign-extend
          push_int((int64_t)x);
          break;
        }
        case 'G': {  // BINFLOAT (big-endian)
          if (!r.read(8, buf)) return fail(FA_ERR_DATA, "truncated BINFLOAT");
          uint64_t x = 0;
          for (int k = 0; k < 8; ++k) x = (x << 8) | buf[k];
          Node n;
          n.t = N_FLOAT;
          std::memcpy(&n.f, &x, 8);
          stack.push_back(add(std::move(n)));
          break;
        }
        case 0x8c:
          if (!rd_u(1, &u) || !push_str((int64_t)u)) return fail(FA_ERR_DATA, "bad SHORT_BINUNICODE");
          break;
        case 'X':
          if (!rd_u(4, &u) || !push_str((int64_t)u)) return fail(FA_ERR_DATA, "bad BINUNICODE");
          break;
        case 0x8d:
          if (!rd_u(8, &u) || !push_str((int64_t)u)) return fail(FA_ERR_DATA, "bad BINUNICODE8");
          break;
        case 'C':
          if (!rd_u(1, &u) || !push_bytes((int64_t)u)) return fail(FA_ERR_DATA, "bad SHORT_BINBYTES");
          break;
        case 'B':
          if (!rd_u(4, &u) || !push_bytes((int64_t)u)) return fail(FA_ERR_DATA, "bad BINBYTES");
          break;
        case 0x8e:
        case 0x96:  // BINBYTES8, BYTEARRAY8 (in-band PickleBuffer)
          if (!rd_u(8, &u) || !push_bytes((int64_t)u)) return fail(FA_ERR_DATA, "bad BINBYTES8");
          break;
        case '}': {
          Node n;
          n.t = N_DICT;
          stack.push_back(add(std::move(n)));
          break;
        }
        case ']': {
          Node n;
          n.t = N_LIST;
          stack.push_back(add(std::move(n)));
          break;
        }
        case ')':
          tuple_of({});
          break;
        case '(':
          marks.push_back(stack.size());
          break;
        case 't': {
          std::vector<int32_t> items;
          if (!pop_mark(&items)) return fail(FA_ERR_DATA, "TUPLE without MARK");
          tuple_of(std::move(items));
          break;
        }
        case 0x85:
          if (!pop(&a)) return fail(FA_ERR_DATA, "TUPLE1 underflow");
          tuple_of({a});
          break;
        case 0x86:
          if (!pop(&b) || !pop(&a)) return fail(FA_ERR_DATA, "TUPLE2 underflow");
          tuple_of({a, b});
          break;
        case 0x87:
          if (!pop(&c) || !pop(&b) || !pop(&a)) return fail(FA_ERR_DATA, "TUPLE3 underflow");
          tuple_of({a, b, c});
          break;
        case 'l':
        case 'd': {
          std::vector<int32_t> items;
          if (!pop_mark(&items)) return fail(FA_ERR_DATA, "LIST/DICT without MARK");
          if (op == 'd' && (items.size() & 1)) return fail(FA_ERR_DATA, "odd DICT items");
          Node n;
          n.t = op == 'l' ? N_LIST : N_DICT;
          n.kids = std::move(items);
          stack.push_back(add(std::move(n)));
          break;
        }
        case 'a':
          if (!pop(&b) || stack.empty()) return fail(FA_ERR_DATA, "APPEND underflow");
          if (nodes[stack.back()].t != N_LIST) return fail(FA_ERR_UNSUPPORTED, "APPEND to a non-list");
          nodes[stack.back()].kids.push_back(b);
          break;
        case 'e': {
          std::vector<int32_t> items;
          if (!pop_mark(&items) || stack.empty()) return fail(FA_ERR_DATA, "APPENDS underflow");
          Node& l = nodes[stack.back()];
          if (l.t != N_LIST) return fail(FA_ERR_UNSUPPORTED, "APPENDS to a non-list");
          l.kids.insert(l.kids.end(), items.begin(), items.end());
          break;
        }
        case 's':
          if (!pop(&b) || !pop(&a) || stack.empty()) return fail(FA_ERR_DATA, "SETITEM underflow");
          if (nodes[stack.back()].t != N_DICT) return fail(FA_ERR_UNSUPPORTED, "SETITEM on a non-dict");
          nodes[stack.back()].kids.push_back(a);
          nodes[stack.back()].kids.push_back(b);
          break;
        case 'u': {
          std::vector<int32_t> items;
          if (!pop_mark(&items) || stack.empty() || (items.size() & 1))
            return fail(FA_ERR_DATA, "SETITEMS underflow");
          Node& d = nodes[stack.back()];
          if (d.t != N_DICT) return fail(FA_ERR_UNSUPPORTED, "SETITEMS on a non-dict");
          d.kids.insert(d.kids.end(), items.begin(), items.end());
          break;
        }
        case 0x94:  // MEMOIZE
          if (stack.empty()) return fail(FA_ERR_DATA, "MEMOIZE on empty stack");
          memo[(int64_t)memo.size()] = stack.back();
          break;
        case 'q':
        case 'r':
          if (!rd_u(op == 'q' ? 1 : 4, &u) || stack.empty()) return fail(FA_ERR_DATA, "bad BINPUT");
          memo[(int64_t)u] = stack.back();
          break;
        case 'h':
        case 'j': {
          if (!rd_u(op == 'h' ? 1 : 4, &u)) return fail(FA_ERR_DATA, "bad BINGET");
          auto it = memo.find((int64_t)u);
          if (it == memo.end()) return fail(FA_ERR_DATA, "BINGET of a missing memo entry");
          stack.push_back(it->second);
          break;
        }
        case 0x93: {  // STACK_GLOBAL
          if (!pop(&b) || !pop(&a)) return fail(FA_ERR_DATA, "STACK_GLOBAL underflow");
          if (nodes[a].t != N_STR || nodes[b].t != N_STR) return fail(FA_ERR_DATA, "STACK_GLOBAL operands");
          if (!allowed_global(nodes[a].s, nodes[b].s))
            return fail(FA_ERR_UNSUPPORTED, "global " + nodes[a].s + "." + nodes[b].s);
          Node n;
          n.t = N_GLOBAL;
          n.s = nodes[a].s;
          n.s2 = nodes[b].s;
          stack.push_back(add(std::move(n)));
          break;
        }
        case 'c': {  // GLOBAL "module\nname\n"
          std::string parts[2];
          for (auto& p : parts) {
            for (int k = 0; k < 256; ++k) {
              if (!r.read(1, buf)) return fail(FA_ERR_DATA, "truncated GLOBAL");
              if (buf[0] == '\n') break;
              p.push_back((char)buf[0]);
            }
          }
          if (!allowed_global(parts[0], parts[1]))
            return fail(FA_ERR_UNSUPPORTED, "global " + parts[0] + "." + parts[1]);
          Node n;
          n.t = N_GLOBAL;
          n.s = parts[0];
          n.s2 = parts[1];
          stack.push_back(add(std::move(n)));
          break;
        }
        case 'R': {  // REDUCE
          if (!pop(&b) || !pop(&a)) return fail(FA_ERR_DATA, "REDUCE underflow");
          if (nodes[a].t != N_GLOBAL || nodes[b].t != N_TUPLE) return fail(FA_ERR_UNSUPPORTED, "REDUCE form");
          if (nodes[a].s == "collections") {  // OrderedDict(): items follow via SETITEMS
            if (!nodes[b].kids.empty()) return fail(FA_ERR_UNSUPPORTED, "OrderedDict with arguments");
            Node n;
            n.t = N_DICT;
            n.ordered = true;
            stack.push_back(add(std::move(n)));
          } else {
            Node n;
            n.t = N_REDUCE;
            n.kids = {a, b};
            stack.push_back(add(std::move(n)));
          }
          break;
        }
        case 'b': {  // BUILD
          if (!pop(&b) || stack.empty()) return fail(FA_ERR_DATA, "BUILD underflow");
          Node& o = nodes[stack.back()];
          if (o.t != N_REDUCE || o.state != -1) return fail(FA_ERR_UNSUPPORTED, "BUILD target");
          o.state = b;
          break;
        }
        case '0':
          if (!pop(&a)) return fail(FA_ERR_DATA, "POP underflow");
          break;
        case '1': {
          std::vector<int32_t> items;
          if (!pop_mark(&items)) return fail(FA_ERR_DATA, "POP_MARK underflow");
          break;
        }
        case '2':
          if (stack.empty()) return fail(FA_ERR_DATA, "DUP underflow");
          stack.push_back(stack.back());
          break;
        default: {
          char m[48];
          std::snprintf(m, sizeof m, "pickle opcode 0x%02x", op);
          return fail(FA_ERR_UNSUPPORTED, m);
        }
      }
    }
    return fail(FA_ERR_DATA, "pickle too long");
  }

  // ---- manifest (JSON) ----
  std::string out;

  bool is_global(int32_t id, const char* name) const {
    const Node& n = nodes[id];
    return n.t == N_GLOBAL && n.s2 == name;
  }
  // numpy dtype node -> "<f4" etc.
  bool dtype_str(int32_t id, std::string* ds) {
    const Node& n = nodes[id];
    if (n.t != N_REDUCE || !is_global(n.kids[0], "dtype")) return false;
    const Node& args = nodes[n.kids[1]];
    if (args.kids.size() != 3 || nodes[args.kids[0]].t != N_STR) return false;
    std::string order = "|";
    if (n.state >= 0) {
      const Node& st = nodes[n.state];
      if (st.t != N_TUPLE || st.kids.size() != 8) return false;
      const Node& ver = nodes[st.kids[0]];
      const Node& bo = nodes[st.kids[1]];
      if (ver.t != N_INT || ver.i != 3 || bo.t != N_STR) return false;
      for (int k = 2; k <= 4; ++k)
        if (nodes[st.kids[k]].t != N_NONE) return false;  // subarray / names / fields
      order = bo.s;
    }
    const std::string& code = nodes[args.kids[0]].s;
    if (code.empty() || code.size() > 8) return false;
    for (char ch : code)
      if (!(std::isalnum((unsigned char)ch))) return false;
    if (code[0] == 'O' || code[0] == 'V' || code[0] == 'U' || code[0] == 'S' || code[0] == 'M' || code[0] == 'm')
      return false;  // object / void / strings / datetimes
    *ds = (order == "=" ? std::string("<") : order) + code;
    return true;
  }
  bool int_tuple(int32_t id, std::vector<int64_t>* v) {
    const Node& n = nodes[id];
    if (n.t != N_TUPLE) return false;
    for (int32_t k : n.kids) {
      if (nodes[k].t != N_INT || nodes[k].i < 0) return false;
      v->push_back(nodes[k].i);
    }
    return true;
  }
  void put_str(const std::string& s) {
    out.push_back('"');
    for (unsigned char ch : s) {
      if (ch == '"' || ch == '\\') {
        out.push_back('\\');
        out.push_back((char)ch);
      } else if (ch < 0x20) {
        char e[8];
        std::snprintf(e, sizeof e, "\\u%04x", ch);
        out += e;
      } else {
        out.push_back((char)ch);
      }
    }
    out.push_back('"');
  }
  void put_i(int64_t v) { out += std::to_string(v); }
  // setstate: ndarray.__setstate__ semantics (protocol <= 4), which converts to native byte order
  void put_nd(const std::string& dt, const std::vector<int64_t>& shape, bool fortran, const Node& data,
              bool setstate) {
    out += "{\"__nd\":[";
    put_str(dt);
    out += ",[";
    for (size_t k = 0; k < shape.size(); ++k) {
      if (k) out.push_back(',');
      put_i(shape[k]);
    }
    out += "],";
    out += fortran ? "true" : "false";
    out.push_back(',');
    put_i(data.off);
    out.push_back(',');
    put_i(data.len);
    out += setstate ? ",1]}" : ",0]}";
  }

  bool emit(int32_t id, int depth) {
    if (depth > 64 || out.size() > kMaxManifest) {
      fail(FA_ERR_UNSUPPORTED, "nesting too deep or manifest too large");
      return false;
    }
    const Node& n = nodes[id];
    switch (n.t) {
      case N_NONE: out += "null"; return true;
      case N_BOOL: out += n.b ? "true" : "false"; return true;
      case N_INT: put_i(n.i); return true;
      case N_FLOAT: {
        char f[40];
        std::snprintf(f, sizeof f, "%a", n.f);
        out += "{\"__f\":\"";
        out += f;
        out += "\"}";
        return true;
      }
      case N_STR: put_str(n.s); return true;
      case N_BYTES:
        out += "{\"__b\":[";
        put_i(n.off);
        out.push_back(',');
        put_i(n.len);
        out += "]}";
        return true;
      case N_TUPLE:
      case N_LIST: {
        out += n.t == N_TUPLE ? "{\"__t\":[" : "[";
        for (size_t k = 0; k < n.kids.size(); ++k) {
          if (k) out.push_back(',');
          if (!emit(n.kids[k], depth + 1)) return false;
        }
        out += n.t == N_TUPLE ? "]}" : "]";
        return true;
      }
      case N_DICT: {
        out += n.ordered ? "{\"__od\":[" : "{\"__d\":[";
        for (size_t k = 0; k < n.kids.size(); k += 2) {
          if (k) out.push_back(',');
          out.push_back('[');
          if (!emit(n.kids[k], depth + 1)) return false;
          out.push_back(',');
          if (!emit(n.kids[k + 1], depth + 1)) return false;
          out.push_back(']');
        }
        out += "]}";
        return true;
      }
      case N_REDUCE: return emit_reduce(n);
      default: fail(FA_ERR_UNSUPPORTED, "bare global as a value"); return false;
    }
  }

  bool emit_reduce(const Node& n) {
    const Node& fn = nodes[n.kids[0]];
    const Node& args = nodes[n.kids[1]];
    std::string dt;
    if (fn.s2 == "_reconstruct") {  // protocol <= 4 ndarray: BUILD(_reconstruct(ndarray, (0,), b'b'), state)
      if (args.kids.size() != 3 || !is_global(args.kids[0], "ndarray") || n.state < 0) goto unsupported;
      {
        const Node& st = nodes[n.state];
        if (st.t != N_TUPLE || st.kids.size() != 5 || nodes[st.kids[0]].t != N_INT || nodes[st.kids[0]].i != 1)
          goto unsupported;
        std::vector<int64_t> shape;
        const Node& fo = nodes[st.kids[3]];
        const Node& data = nodes[st.kids[4]];
        if (!int_tuple(st.kids[1], &shape) || !dtype_str(st.kids[2], &dt) || fo.t != N_BOOL || data.t != N_BYTES)
          goto unsupported;
        put_nd(dt, shape, fo.b, data, true);
        return true;
      }
    }
    if (fn.s2 == "_frombuffer") {  // protocol 5 ndarray: _frombuffer(buffer, dtype, shape, order)
      if (args.kids.size() != 4 || n.state >= 0) goto unsupported;
      {
        std::vector<int64_t> shape;
        const Node& data = nodes[args.kids[0]];
        const Node& order = nodes[args.kids[3]];
        if (data.t != N_BYTES || !dtype_str(args.kids[1], &dt) || !int_tuple(args.kids[2], &shape) ||
            order.t != N_STR)
          goto unsupported;
        put_nd(dt, shape, order.s == "F", data, false);
        return true;
      }
    }
    if (fn.s2 == "scalar") {  // numpy scalar: scalar(dtype, bytes)
      if (args.kids.size() != 2 || n.state >= 0 || nodes[args.kids[1]].t != N_BYTES ||
          !dtype_str(args.kids[0], &dt))
        goto unsupported;
      const Node& data = nodes[args.kids[1]];
      out += "{\"__sc\":[";
      put_str(dt);
      out.push_back(',');
      put_i(data.off);
      out.push_back(',');
      put_i(data.len);
      out += "]}";
      return true;
    }
    if (fn.s2 == "dtype" && dtype_str((int32_t)(&n - nodes.data()), &dt)) {
      out += "{\"__dt\":";
      put_str(dt);
      out += "}";
      return true;
    }
  unsupported:
    fail(FA_ERR_UNSUPPORTED, "unsupported reduce " + fn.s + "." + fn.s2);
    return false;
  }
};

}  // namespace

extern "C" {

const char* fa_wire_last_error(void) { return g_wire_error.c_str(); }

int64_t fa_b64_decoded_size(const char* src, int64_t n) {
  B64 b(src, n);
  if (!b.ok) return wfail(FA_ERR_DATA, "not canonical base64 (length or padding)");
  return b.total;
}

int fa_b64_decode(const char* src, int64_t n, uint8_t* dst, int64_t cap, int32_t threads) {
  B64 b(src, n);
  if (!b.ok) return wfail(FA_ERR_DATA, "not canonical base64 (length or padding)");
  if (b.total > cap || (b.total && !dst)) return wfail(FA_ERR_ARG, "output buffer too small");
  const int64_t tasks = (b.total + kPiece - 1) / kPiece;
  std::atomic<int> bad{0};
  Pool::get().run(tasks, clamp_threads(threads), [&](int64_t t) {
    const int64_t o = t * kPiece, len = o + kPiece < b.total ? kPiece : b.total - o;
    if (!b.range(o, len, dst + o)) bad.store(1);
  });
  return bad.load() ? wfail(FA_ERR_DATA, "non-alphabet character in base64 input") : FA_OK;
}

int fa_b64_decode_ranges(const char* src, int64_t n, int32_t count, const int64_t* offsets,
                         const int64_t* lengths, void* const* dsts, int32_t threads) {
  B64 b(src, n);
  if (!b.ok) return wfail(FA_ERR_DATA, "not canonical base64 (length or padding)");
  if (count < 0 || (count && (!offsets || !lengths || !dsts))) return wfail(FA_ERR_ARG, "bad range arrays");
  std::vector<int64_t> first(count + 1, 0);  // task index of each range's first piece
  for (int32_t r = 0; r < count; ++r) {
    if (offsets[r] < 0 || lengths[r] < 0 || offsets[r] + lengths[r] > b.total || (lengths[r] && !dsts[r]))
      return wfail(FA_ERR_ARG, "range outside the decoded payload");
    first[r + 1] = first[r] + (lengths[r] + kPiece - 1) / kPiece;
  }
  std::atomic<int> bad{0};
  Pool::get().run(first[count], clamp_threads(threads), [&](int64_t t) {
    int32_t lo = 0, hi = count;  // range r with first[r] <= t < first[r+1]
    while (hi - lo > 1) {
      const int32_t mid = (lo + hi) / 2;
      if (first[mid] <= t) lo = mid; else hi = mid;
    }
    const int64_t p = (t - first[lo]) * kPiece;
    const int64_t len = p + kPiece < lengths[lo] ? kPiece : lengths[lo] - p;
    if (!b.range(offsets[lo] + p, len, static_cast<uint8_t*>(dsts[lo]) + p)) bad.store(1);
  });
  return bad.load() ? wfail(FA_ERR_DATA, "non-alphabet character in base64 input") : FA_OK;
}

namespace {
// the last 1-2 bytes of an encode, with '=' padding (what base64.b64encode emits)
void enc_tail(const uint8_t* s, int64_t rem, char* d) {
  const uint32_t v = ((uint32_t)s[0] << 16) | (rem == 2 ? (uint32_t)s[1] << 8 : 0);
  d[0] = kAlpha[(v >> 18) & 63];
  d[1] = kAlpha[(v >> 12) & 63];
  d[2] = rem == 2 ? kAlpha[(v >> 6) & 63] : '=';
  d[3] = '=';
}
}  // namespace

int fa_b64_encode(const uint8_t* src, int64_t n, char* dst, int64_t cap, int32_t threads) {
  if (n < 0 || (n && !src)) return wfail(FA_ERR_ARG, "bad input");
  const int64_t ng = n / 3, rem = n % 3, outn = 4 * ((n + 2) / 3);
  if (cap < outn || (outn && !dst)) return wfail(FA_ERR_ARG, "output buffer too small");
  const int64_t per = kPiece / 3;  // groups per task
  const int64_t tasks = (ng + per - 1) / per;
  Pool::get().run(tasks, clamp_threads(threads), [&](int64_t t) {
    const int64_t g0 = t * per, g1 = g0 + per < ng ? g0 + per : ng;
    enc_groups(src + 3 * g0, g1 - g0, dst + 4 * g0);
  });
  if (rem) enc_tail(src + 3 * ng, rem, dst + 4 * ng);
  return FA_OK;
}

int fa_b64_encode_gather(int32_t count, const uint8_t* const* srcs, const int64_t* lens, char* dst,
                         int64_t cap, int32_t threads) {
  if (count < 0 || (count && (!srcs || !lens))) return wfail(FA_ERR_ARG, "bad chunk arrays");
  std::vector<int64_t> off(count + 1, 0);
  for (int32_t i = 0; i < count; ++i) {
    if (lens[i] < 0 || (lens[i] && !srcs[i])) return wfail(FA_ERR_ARG, "bad chunk");
    off[i + 1] = off[i] + lens[i];
  }
  const int64_t n = off[count], ng = n / 3, rem = n % 3, outn = 4 * ((n + 2) / 3);
  if (cap < outn || (outn && !dst)) return wfail(FA_ERR_ARG, "output buffer too small");
  // byte position (chunk c, offset o) of decoded byte b: the last chunk starting at or before b
  auto locate = [&](int64_t b, int32_t& c, int64_t& o) {
    c = (int32_t)(std::upper_bound(off.begin(), off.end(), b) - off.begin()) - 1;
    o = b - off[c];
  };
  auto take = [&](int32_t& c, int64_t& o, uint8_t* out, int64_t cnt) {  // across chunk ends
    for (int64_t j = 0; j < cnt; ++j) {
      while (o == lens[c]) { ++c; o = 0; }
      out[j] = srcs[c][o++];
    }
  };
  const int64_t per = kPiece / 3;
  const int64_t tasks = (ng + per - 1) / per;
  Pool::get().run(tasks, clamp_threads(threads), [&](int64_t t) {
    int64_t g = t * per;
    const int64_t g1 = g + per < ng ? g + per : ng;
    int32_t c;
    int64_t o;
    locate(3 * g, c, o);
    char* d = dst + 4 * g;
    while (g < g1) {
      while (o == lens[c]) { ++c; o = 0; }
      int64_t whole = (lens[c] - o) / 3;
      if (whole > g1 - g) whole = g1 - g;
      if (whole > 0) {  // groups inside one chunk
        enc_groups(srcs[c] + o, whole, d);
        g += whole, o += 3 * whole, d += 4 * whole;
        continue;
      }
      uint8_t tmp[3];  // a group straddling chunk ends
      take(c, o, tmp, 3);
      enc_groups(tmp, 1, d);
      ++g, d += 4;
    }
  });
  if (rem) {
    uint8_t tmp[2];
    int32_t c;
    int64_t o;
    locate(3 * ng, c, o);
    take(c, o, tmp, rem);
    enc_tail(tmp, rem, dst + 4 * ng);
  }
  return FA_OK;
}

int fa_pickle_scan_b64(const char* src, int64_t n, char* out, int64_t cap, int64_t* out_len) {
  if (!out_len) return wfail(FA_ERR_ARG, "out_len is NULL");
  B64 b(src, n);
  if (!b.ok) return wfail(FA_ERR_DATA, "not canonical base64 (length or padding)");
  Scanner sc;
  B64Reader r(b);
  int rc = sc.run(r);
  if (rc == FA_OK && r.pos != b.total) rc = sc.fail(FA_ERR_DATA, "bytes after STOP");
  if (rc == FA_OK && !sc.emit(sc.stack.back(), 0)) rc = sc.err;
  if (rc != FA_OK) return wfail(rc, sc.why.c_str());
  *out_len = (int64_t)sc.out.size();
  if (!out || cap < (int64_t)sc.out.size()) return wfail(FA_ERR_SIZE, "manifest buffer too small");
  std::memcpy(out, sc.out.data(), sc.out.size());
  return FA_OK;
}

int fa_pickle_scan(const uint8_t* buf, int64_t n, char* out, int64_t cap, int64_t* out_len) {
  if (!out_len || n < 0 || (n && !buf)) return wfail(FA_ERR_ARG, "bad arguments");
  Scanner sc;
  MemReader r{buf, n};
  int rc = sc.run(r);
  if (rc == FA_OK && r.pos != n) rc = sc.fail(FA_ERR_DATA, "bytes after STOP");
  if (rc == FA_OK && !sc.emit(sc.stack.back(), 0)) rc = sc.err;
  if (rc != FA_OK) return wfail(rc, sc.why.c_str());
  *out_len = (int64_t)sc.out.size();
  if (!out || cap < (int64_t)sc.out.size()) return wfail(FA_ERR_SIZE, "manifest buffer too small");
  std::memcpy(out, sc.out.data(), sc.out.size());
  return FA_OK;
}

}  // extern "C"
