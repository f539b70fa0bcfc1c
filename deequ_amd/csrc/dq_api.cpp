// dq_api.cpp -- host side of the deequ_amd C-ABI (include/deequ_amd.h).
//
// Plays the role of AnalysisRunner.runScanningAnalyzers (runners/AnalysisRunner.scala:289-336)
// for GPU-eligible analyzers: it groups the requested analyzers into fused scan tasks (one
// per (column, where) pair, Compliance predicates riding along), HLL tasks and predicate
// mask programs, launches one fused pass per batch, and maps the device aggregates back to
// the exact Scala State values (fromAggregationResult in Size/Completeness/Compliance/Sum/
// Mean/StandardDeviation/Minimum/Maximum/ApproxCountDistinct .scala) including Spark's NULL
// -> None rules.  It also implements the State algebra (State.sum / metricValue) so GPU
// states from several devices merge exactly like Spark partial states.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#include "dq_internal.h"
#include "dq_keypack.h"
#include "dq_uuidpack.h"
#include "dq_numparse.h"
#include "dq_predeval.h"
#include "../../include/deequ_amd_diag.h"
#include "hll_p9_tables.h"

using namespace dq;

// ------------------------------------------------------------------------------ errors
static thread_local std::string g_last_error;

static dq_status fail(dq_status s, const std::string& msg) {
  g_last_error = msg;
  return s;
}

#define DQ_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(e_ == hipErrorOutOfMemory ? DQ_ERR_OOM : DQ_ERR_DEVICE,              \
                  std::string(#expr) + " failed: " + hipGetErrorString(e_));           \
  } while (0)

#define DQ_TRY(expr)                 \
  do {                               \
    dq_status s_ = (expr);           \
    if (s_ != DQ_OK) return s_;      \
  } while (0)

extern "C" const char* dq_last_error(void) { return g_last_error.c_str(); }
extern "C" int dq_abi_version(void) { return DQ_ABI_VERSION; }

// ------------------------------------------------------------------------------ helpers
static int type_size(int t) {
  switch (t) {
    case DQ_T_INT8: return 1;
    case DQ_T_INT16: return 2;
    case DQ_T_INT32: return 4;
    case DQ_T_INT64: return 8;
    case DQ_T_FLOAT32: return 4;
    case DQ_T_FLOAT64: return 8;
    default: return 0;  // BOOL (bits), UTF8 (variable)
  }
}
static bool is_numeric(int t) { return t >= DQ_T_INT8 && t <= DQ_T_FLOAT64; }
static bool is_integral(int t) { return t >= DQ_T_INT8 && t <= DQ_T_INT64; }
static bool valid_type(int t) { return t >= DQ_T_BOOL && t <= DQ_T_UTF8; }

// Device block pool.  hipMalloc / hipFree of multi-GB buffers cost milliseconds to seconds, and
// every hipFree synchronises the device -- a profiler run creates and drops dozens of small
// tables and plans, each free a device-wide stall.  Freed blocks are therefore kept per device
// and handed out again (best fit within 2x of the request).  A block may still be in use by a
// stream when it is freed: it is reused only after a device synchronisation (taken outside the
// pool's lock; one sync fences every block released before it began).  On an allocation
// failure the device's cached blocks are released and the allocation retried.
class BlockPool {
 public:
  static constexpr size_t kPoolMin = 0;  // every block (DevBuf rounds requests up to 256 B)
  static constexpr size_t kPoolMaxCached = (size_t)128 << 30;

  static BlockPool& get() {
    static BlockPool* pool = new BlockPool();  // never destroyed: no hipFree after runtime teardown
    return *pool;
  }

  hipError_t alloc(int dev, size_t bytes, void** out) {
    if (bytes >= kPoolMin) {
      std::unique_lock<std::mutex> g(mu_);
      int best = -1;
      for (size_t i = 0; i < blocks_.size(); ++i) {
        const Blk& b = blocks_[i];
        if (b.dev == dev && b.bytes >= bytes && b.bytes <= 2 * bytes &&
            (best < 0 || b.bytes < blocks_[best].bytes))
          best = (int)i;
      }
      if (best >= 0) {
        // claim the block, then (if work on it may still be queued) synchronise the device
        // OUTSIDE the lock: other threads' allocations and releases proceed meanwhile (the
        // profiler runs several group-bys on their own streams at once)
        const Blk blk = blocks_[best];
        cached_ -= blk.bytes;
        blocks_.erase(blocks_.begin() + best);
        if (!blk.fenced) {
          const uint64_t upto = seq_;  // every block released so far is fenced by this sync
          g.unlock();
          hipError_t e = hipDeviceSynchronize();
          g.lock();
          if (e != hipSuccess) {
            blocks_.push_back(blk);
            cached_ += blk.bytes;
            return e;
          }
          for (Blk& b : blocks_)
            if (b.dev == dev && b.seq <= upto) b.fenced = true;
        }
        *out = blk.ptr;
        return hipSuccess;
      }
    }
    hipError_t e = hipMalloc(out, bytes);
    if (e == hipErrorOutOfMemory) {
      (void)hipGetLastError();
      trim(dev);
      e = hipMalloc(out, bytes);
    }
    return e;
  }

  void release(int dev, void* ptr, size_t bytes) {
    if (bytes < kPoolMin) {
      (void)hipFree(ptr);
      return;
    }
    std::lock_guard<std::mutex> g(mu_);
    blocks_.push_back(Blk{ptr, bytes, dev, false, ++seq_});
    cached_ += bytes;
    while (cached_ > kPoolMaxCached && !blocks_.empty()) {  // drop the oldest
      cached_ -= blocks_.front().bytes;
      (void)hipFree(blocks_.front().ptr);
      blocks_.erase(blocks_.begin());
    }
  }

  void trim(int dev) {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < blocks_.size();) {
      if (blocks_[i].dev == dev) {
        cached_ -= blocks_[i].bytes;
        (void)hipFree(blocks_[i].ptr);
        blocks_.erase(blocks_.begin() + i);
      } else {
        ++i;
      }
    }
  }

 private:
  struct Blk {
    void* ptr;
    size_t bytes;
    int dev;
    bool fenced;
    uint64_t seq;  // release order
  };
  std::mutex mu_;
  std::vector<Blk> blocks_;
  size_t cached_ = 0;
  uint64_t seq_ = 0;
};

// Streams and pinned host blocks are recycled too: the profiler creates dozens of plans and
// frequency tables per run, and hipStreamCreate / hipStreamDestroy / hipHostMalloc each cost
// the host up to a millisecond (measured: ~1 ms host gaps before every table in a C5 trace).
static bool getenv_flag(const char* name) {  // test knobs: set and not "0"
  const char* e = std::getenv(name);
  return e && e[0] && e[0] != '0';
}

class StreamPool {
 public:
  static StreamPool& get() {
    static StreamPool* pool = new StreamPool();  // never destroyed (runtime teardown order)
    return *pool;
  }
  hipError_t acquire(int dev, hipStream_t* out) {
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i = 0; i < free_.size(); ++i) {
        if (free_[i].first == dev) {
          *out = free_[i].second;
          free_.erase(free_.begin() + i);
          return hipSuccess;
        }
      }
    }
    return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
  }
  void release(int dev, hipStream_t s) {  // after the owner's last work on it completed
    if (!s) return;
    (void)hipStreamSynchronize(s);
    std::lock_guard<std::mutex> g(mu_);
    if (free_.size() >= 64) {
      (void)hipStreamDestroy(s);
      return;
    }
    free_.emplace_back(dev, s);
  }

 private:
  std::mutex mu_;
  std::vector<std::pair<int, hipStream_t>> free_;
};

class PinnedPool {
 public:
  static PinnedPool& get() {
    static PinnedPool* pool = new PinnedPool();
    return *pool;
  }
  hipError_t alloc(size_t bytes, void** out) {
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i = 0; i < free_.size(); ++i) {
        if (free_[i].second >= bytes && free_[i].second <= 4 * bytes + 4096) {
          *out = free_[i].first;
          sizes_[*out] = free_[i].second;
          free_.erase(free_.begin() + i);
          return hipSuccess;
        }
      }
    }
    const size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipHostMalloc(out, want, hipHostMallocDefault);
    if (e == hipSuccess) {
      std::lock_guard<std::mutex> g(mu_);
      sizes_[*out] = want;
    }
    return e;
  }
  void release(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(mu_);
    auto it = sizes_.find(p);
    const size_t n = it == sizes_.end() ? 0 : it->second;
    if (it != sizes_.end()) sizes_.erase(it);
    if (free_.size() >= 64 || n == 0) {
      (void)hipHostFree(p);
      return;
    }
    free_.emplace_back(p, n);
  }

 private:
  std::mutex mu_;
  std::vector<std::pair<void*, size_t>> free_;
  std::unordered_map<void*, size_t> sizes_;
};

struct DevBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  int dev = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept { swap(o); }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      swap(o);
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void swap(DevBuf& o) noexcept {
    std::swap(ptr, o.ptr);
    std::swap(cap, o.cap);
    std::swap(dev, o.dev);
  }
  void release() {
    if (ptr) BlockPool::get().release(dev, ptr, cap);
    ptr = nullptr;
    cap = 0;
  }
  dq_status ensure(size_t bytes) {
    if (bytes <= cap) return DQ_OK;
    release();
    size_t want = std::max<size_t>(bytes, 256);
    want = (want + 255) & ~(size_t)255;  // padded: kernels may read whole aligned words
    DQ_HIP(hipGetDevice(&dev));
    DQ_HIP(BlockPool::get().alloc(dev, want, &ptr));
    cap = want;
    return DQ_OK;
  }
};

struct dq_ctx {
  int device = 0;
};

extern "C" dq_status dq_release_cached_memory(int device) {
  BlockPool::get().trim(device);
  return DQ_OK;
}

// ------------------------------------------------------------------------------ diagnostics
extern "C" dq_status dq_diag_hash_rate(int device, int with_hll, int reps, double* hashes_per_sec) {
  if (!hashes_per_sec || reps < 1) return fail(DQ_ERR_INVALID, "hashes_per_sec is NULL or reps < 1");
  DQ_HIP(hipSetDevice(device));
  hipDeviceProp_t p;
  DQ_HIP(hipGetDeviceProperties(&p, device));
  const int blocks = p.multiProcessorCount * 8;  // 8 workgroups (32 waves) per CU
  const int iters = 4096;                          // 4 chains -> 16384 hashes per lane
  void* sink = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipMalloc(&sink, sizeof(uint64_t));
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = launch_diag_hash(blocks, 64, with_hll != 0, static_cast<uint64_t*>(sink), st);  // warm-up
  float best = 0.f;
  for (int r = 0; r < reps && e == hipSuccess; ++r) {
    e = hipEventRecord(e0, st);
    if (e == hipSuccess) e = launch_diag_hash(blocks, iters, with_hll != 0, static_cast<uint64_t*>(sink), st);
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess && (best == 0.f || ms < best)) best = ms;
  }
  if (st) (void)hipStreamSynchronize(st);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (sink) (void)hipFree(sink);
  if (e != hipSuccess) return fail(DQ_ERR_DEVICE, std::string("dq_diag_hash_rate: ") + hipGetErrorString(e));
  *hashes_per_sec = (double)blocks * kBlock * 4.0 * iters / (best * 1e-3);
  return DQ_OK;
}

extern "C" dq_status dq_diag_table_hash(int device, const uint64_t* k0, const uint64_t* k1, const uint32_t* len,
                                        int64_t n, uint64_t* out) {
  if (n < 0 || (n > 0 && (!k0 || !k1 || !len || !out))) return fail(DQ_ERR_INVALID, "bad argument");
  if (n == 0) return DQ_OK;
  DQ_HIP(hipSetDevice(device));
  void* d = nullptr;
  const size_t bytes = (size_t)n * (8 + 8 + 4 + 16);
  DQ_HIP(hipMalloc(&d, bytes));
  uint8_t* b = static_cast<uint8_t*>(d);
  uint64_t* d_k0 = reinterpret_cast<uint64_t*>(b);
  uint64_t* d_k1 = d_k0 + n;
  uint64_t* d_out = d_k1 + n;
  uint32_t* d_len = reinterpret_cast<uint32_t*>(d_out + 2 * n);
  hipError_t e = hipMemcpy(d_k0, k0, n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_k1, k1, n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_len, len, n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_freq_hash(d_k0, d_k1, d_len, n, d_out, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, d_out, n * 16, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(DQ_ERR_DEVICE, std::string("dq_diag_table_hash: ") + hipGetErrorString(e));
  return DQ_OK;
}

extern "C" dq_status dq_device_count(int* out) {
  if (!out) return fail(DQ_ERR_INVALID, "out is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  int gfx950 = 0;
  for (int d = 0; d < n; ++d) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0)
      ++gfx950;
  }
  *out = gfx950;
  return DQ_OK;
}

extern "C" dq_status dq_ctx_create(int device, int flags, dq_ctx** out) {
  (void)flags;
  if (!out) return fail(DQ_ERR_INVALID, "out is NULL");
  *out = nullptr;
  int n = 0;
  DQ_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(DQ_ERR_INVALID, "device index out of range");
  hipDeviceProp_t p;
  DQ_HIP(hipGetDeviceProperties(&p, device));
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
    return fail(DQ_ERR_DEVICE, std::string("device is not gfx950 (MI355X): ") + p.gcnArchName);
  dq_ctx* c = new dq_ctx();
  c->device = device;
  *out = c;
  return DQ_OK;
}

extern "C" dq_status dq_ctx_destroy(dq_ctx* ctx) {
  delete ctx;
  return DQ_OK;
}

// ------------------------------------------------------------------------------ predicates
// Value types of the validator.  V_F32 is a FloatType value (a FLOAT32 column or a cast to
// FLOAT32; the device holds it as the fp64 of the same value); V_NULL the untyped NULL literal,
// compatible with every type (Spark types it by the other side).
enum VT { V_INT = 0, V_FLT = 1, V_BOOL = 2, V_STR = 3, V_F32 = 4, V_NULL = 5 };

struct Program {
  std::vector<PredInsn> code;
  std::vector<int> columns;  // referenced batch columns (sorted, unique)
  std::string pool;          // string literals (DQ_P_LIT_STRING), offsets relative to this
  std::string key;           // byte image for de-duplication
};

static bool vt_fractional(int t) { return t == V_FLT || t == V_F32; }

// The binary-operand rules of the header's "Type rules" (include/deequ_amd.h): a pair the IR
// cannot evaluate exactly as Spark 2.2 would is DQ_ERR_UNSUPPORTED.
static dq_status check_pair(int a, int b, const char* what) {
  if (a == V_NULL || b == V_NULL) return DQ_OK;
  if ((a == V_STR) != (b == V_STR))  // Spark casts the string: only DQ_P_CAST_DOUBLE does that
    return fail(DQ_ERR_UNSUPPORTED, std::string(what) + " of a string with a non-string");
  if ((a == V_F32 && b == V_INT) || (a == V_INT && b == V_F32))
    return fail(DQ_ERR_UNSUPPORTED, std::string(what) + " of a FloatType value with an integral value: Spark "
                "compares in FloatType, so the integral side needs a DQ_P_CAST to FLOAT32");
  return DQ_OK;
}

static dq_status validate_predicate(const dq_predicate& p, const int32_t* types, int n_cols,
                                    Program* out) {
  if (!p.code || p.n_insns <= 0) return fail(DQ_ERR_INVALID, "empty predicate");
  if (p.n_insns > 256) return fail(DQ_ERR_UNSUPPORTED, "predicate too long");
  std::vector<int> st;  // value types
  Program prog;
  for (int i = 0; i < p.n_insns; ++i) {
    const dq_pred_insn& in = p.code[i];
    PredInsn pi{in.opcode, in.arg, in.i64, in.f64};
    switch (in.opcode) {
      case DQ_P_COLUMN: {
        if (in.arg < 0 || in.arg >= n_cols) return fail(DQ_ERR_INVALID, "predicate column out of range");
        const int t = types[in.arg];
        st.push_back(t == DQ_T_UTF8 ? V_STR : t == DQ_T_BOOL ? V_BOOL : t == DQ_T_FLOAT32 ? V_F32
                     : (is_integral(t) ? V_INT : V_FLT));
        prog.columns.push_back(in.arg);
        break;
      }
      case DQ_P_LIT_STRING: {
        if (in.i64 < 0 || in.arg < 0 || (in.arg > 0 && !p.strings) || in.i64 + in.arg > (int64_t)p.strings_len)
          return fail(DQ_ERR_INVALID, "string literal outside the predicate's string pool");
        st.push_back(V_STR);
        break;
      }
      case DQ_P_LIT_INT: st.push_back(V_INT); break;
      case DQ_P_LIT_FLOAT: st.push_back(V_FLT); break;
      case DQ_P_LIT_NULL: st.push_back(V_NULL); break;
      case DQ_P_CAST_DOUBLE:  // Cast(-> DoubleType) of a string or a number
        if (st.empty()) return fail(DQ_ERR_INVALID, "predicate stack underflow");
        if (st.back() == V_BOOL) return fail(DQ_ERR_UNSUPPORTED, "cast of a boolean to double");
        if (st.back() != V_NULL) st.back() = V_FLT;
        break;
      case DQ_P_CAST: {  // Cast(numeric / boolean -> arg)
        if (st.empty()) return fail(DQ_ERR_INVALID, "predicate stack underflow");
        const int to = in.arg;
        int vt;
        switch (to) {
          case DQ_T_INT8: case DQ_T_INT16: case DQ_T_INT32: case DQ_T_INT64: vt = V_INT; break;
          case DQ_T_FLOAT32: vt = V_F32; break;
          case DQ_T_FLOAT64: vt = V_FLT; break;
          case DQ_T_BOOL: vt = V_BOOL; break;
          default:
            return fail(DQ_ERR_UNSUPPORTED, "DQ_P_CAST to type " + std::to_string(to) +
                        " (only INT8..INT64, FLOAT32, FLOAT64 and BOOL are evaluated on the GPU)");
        }
        if (st.back() == V_STR)
          return fail(DQ_ERR_UNSUPPORTED, "DQ_P_CAST of a string (Spark's UTF8String casts stay on Spark)");
        if (st.back() != V_NULL) st.back() = vt;
        break;
      }
      case DQ_P_TRUE: case DQ_P_FALSE: st.push_back(V_BOOL); break;
      case DQ_P_COALESCE: {
        if (st.size() < 2) return fail(DQ_ERR_INVALID, "predicate stack underflow");
        const int b = st.back(); st.pop_back();
        const int a = st.back(); st.pop_back();
        if (a != V_NULL && b != V_NULL && (a == V_BOOL) != (b == V_BOOL))
          return fail(DQ_ERR_UNSUPPORTED, "COALESCE of mixed boolean/numeric");
        DQ_TRY(check_pair(a, b, "COALESCE"));
        int r;
        if (a == V_NULL) r = b;
        else if (b == V_NULL) r = a;
        else if (a == V_FLT || b == V_FLT) r = V_FLT;
        else if (a == V_F32 || b == V_F32) r = V_F32;  // (F32, F32): the device keeps the value
        else r = a;
        st.push_back(r);
        break;
      }
      case DQ_P_EQ: case DQ_P_NE: case DQ_P_LT: case DQ_P_LE: case DQ_P_GT: case DQ_P_GE:
      case DQ_P_EQ_NULLSAFE: {
        if (st.size() < 2) return fail(DQ_ERR_INVALID, "predicate stack underflow");
        const int b = st.back(); st.pop_back();
        const int a = st.back(); st.pop_back();
        if (in.arg != DQ_CMP_AS_INT64 && in.arg != DQ_CMP_AS_FLOAT64)
          return fail(DQ_ERR_INVALID, "comparison type must be DQ_CMP_AS_INT64 or DQ_CMP_AS_FLOAT64");
        if (in.arg == DQ_CMP_AS_INT64 && (vt_fractional(a) || vt_fractional(b)))
          return fail(DQ_ERR_UNSUPPORTED, "int64 comparison of a floating-point operand (Spark compares "
                      "that pair in a fractional type: cast it or compare as DQ_CMP_AS_FLOAT64)");
        DQ_TRY(check_pair(a, b, "comparison"));
        st.push_back(V_BOOL);
        break;
      }
      case DQ_P_IS_NULL: case DQ_P_IS_NOT_NULL:
        if (st.empty()) return fail(DQ_ERR_INVALID, "predicate stack underflow");
        st.back() = V_BOOL;
        break;
      case DQ_P_NOT:
        if (st.empty() || st.back() != V_BOOL) return fail(DQ_ERR_INVALID, "NOT of a non-boolean");
        break;
      case DQ_P_AND: case DQ_P_OR: {
        if (st.size() < 2) return fail(DQ_ERR_INVALID, "predicate stack underflow");
        const int b = st.back(); st.pop_back();
        const int a = st.back(); st.pop_back();
        if (a != V_BOOL || b != V_BOOL) return fail(DQ_ERR_INVALID, "AND/OR of a non-boolean");
        st.push_back(V_BOOL);
        break;
      }
      default:
        return fail(DQ_ERR_UNSUPPORTED, "unknown predicate opcode " + std::to_string(in.opcode));
    }
    if ((int)st.size() > kMaxStack) return fail(DQ_ERR_UNSUPPORTED, "predicate stack too deep");
    prog.code.push_back(pi);
  }
  if (st.size() != 1 || st.back() != V_BOOL)
    return fail(DQ_ERR_INVALID, "predicate must leave exactly one boolean");
  std::sort(prog.columns.begin(), prog.columns.end());
  prog.columns.erase(std::unique(prog.columns.begin(), prog.columns.end()), prog.columns.end());
  if (p.strings && p.strings_len > 0) prog.pool.assign(reinterpret_cast<const char*>(p.strings), p.strings_len);
  prog.key.assign(reinterpret_cast<const char*>(prog.code.data()), prog.code.size() * sizeof(PredInsn));
  prog.key += prog.pool;
  if (out) *out = std::move(prog);
  return DQ_OK;
}

static int cmp_of(int opcode) {
  switch (opcode) {
    case DQ_P_EQ: return CMP_EQ;
    case DQ_P_NE: return CMP_NE;
    case DQ_P_LT: return CMP_LT;
    case DQ_P_LE: return CMP_LE;
    case DQ_P_GT: return CMP_GT;
    case DQ_P_GE: return CMP_GE;
    case DQ_P_EQ_NULLSAFE: return CMP_EQNS;
    default: return -1;
  }
}
// Derive the branch-free selectors of FastPred (see dq_internal.h) from kind / op.
static void finalize_fast_pred(FastPred* fp) {
  const uint32_t ON = ~0u;
  fp->m_lt = fp->m_eq = fp->m_gt = 0;
  fp->f_cmp = fp->f_coal = fp->f_isnull = fp->f_isnotnull = fp->f_true = fp->f_mask = 0;
  fp->f_nn_valid = fp->f_nn_one = fp->cmp_sel = 0;
  switch (fp->kind) {
    case FP_CMP:
    case FP_COALESCE_CMP:
      fp->f_cmp = ON;
      if (fp->kind == FP_COALESCE_CMP) {
        fp->f_coal = ON;
        fp->f_nn_one = ON;
      } else {
        fp->f_nn_valid = ON;
      }
      switch (fp->op) {
        case CMP_EQ: fp->m_eq = ON; break;
        case CMP_NE: fp->m_lt = fp->m_gt = ON; break;
        case CMP_LT: fp->m_lt = ON; break;
        case CMP_LE: fp->m_lt = fp->m_eq = ON; break;
        case CMP_GT: fp->m_gt = ON; break;
        default: fp->m_gt = fp->m_eq = ON; break;  // CMP_GE
      }
      if (!(fp->as_f64 && fp->lit_f != fp->lit_f)) {  // a NaN literal keeps the three masks
        switch (fp->op) {
          case CMP_EQ: fp->cmp_sel = CS_EQ; break;
          case CMP_NE: fp->cmp_sel = CS_EQ | CS_INV; break;
          case CMP_LT: fp->cmp_sel = CS_LT; break;
          case CMP_LE: fp->cmp_sel = CS_LE; break;
          case CMP_GT: fp->cmp_sel = CS_LE | CS_INV; break;
          case CMP_GE: fp->cmp_sel = CS_LT | CS_INV; break;
          default: break;
        }
      }
      break;
    case FP_IS_NULL: fp->f_isnull = ON; fp->f_nn_one = ON; break;
    case FP_IS_NOT_NULL: fp->f_isnotnull = ON; fp->f_nn_one = ON; break;
    case FP_CONST:
      if (fp->lit_i == 1) fp->f_true = ON;
      if (fp->lit_i != -1) fp->f_nn_one = ON;
      break;
    case FP_MASK: fp->f_mask = ON; break;
    default: break;
  }
}

static int flip_cmp(int c) {
  switch (c) {
    case CMP_LT: return CMP_GT;
    case CMP_LE: return CMP_GE;
    case CMP_GT: return CMP_LT;
    case CMP_GE: return CMP_LE;
    default: return c;
  }
}

// Recognise the forms the fused kernel evaluates inline on its primary column.  Returns the
// referenced column (or -2 for a column-free constant) when `fp` was filled, else -1.
static int fast_form(const Program& prog, const int32_t* types, FastPred* fp) {
  const auto& c = prog.code;
  std::memset(fp, 0, sizeof(*fp));
  auto lit_ok = [](const PredInsn& in) { return in.opcode == DQ_P_LIT_INT || in.opcode == DQ_P_LIT_FLOAT; };
  auto set_lit = [](const PredInsn& in, bool as_f64, int64_t* li, double* lf) -> bool {
    if (as_f64) {
      *lf = in.opcode == DQ_P_LIT_FLOAT ? in.f64 : (double)in.i64;
      return true;
    }
    if (in.opcode != DQ_P_LIT_INT) return false;
    *li = in.i64;
    return true;
  };
  auto numeric_col = [&](const PredInsn& in) { return in.opcode == DQ_P_COLUMN && is_numeric(types[in.arg]); };
  if (c.size() == 1 && (c[0].opcode == DQ_P_TRUE || c[0].opcode == DQ_P_FALSE)) {
    fp->kind = FP_CONST;
    fp->lit_i = c[0].opcode == DQ_P_TRUE ? 1 : 0;
    return -2;
  }
  if (c.size() == 1 && c[0].opcode == DQ_P_COLUMN && types[c[0].arg] == DQ_T_BOOL) {
    // a boolean column as the predicate (`where b`, profiler pass-3 histograms): counted from
    // the value and validity bitmaps by the bits scan, no predicate kernel
    fp->kind = FP_BOOL;
    return c[0].arg;
  }
  if (c.size() == 2 && c[0].opcode == DQ_P_COLUMN &&
      (c[1].opcode == DQ_P_IS_NULL || c[1].opcode == DQ_P_IS_NOT_NULL)) {
    fp->kind = c[1].opcode == DQ_P_IS_NULL ? FP_IS_NULL : FP_IS_NOT_NULL;
    return c[0].arg;
  }
  if (c.size() == 3 && cmp_of(c[2].opcode) >= 0 && c[2].opcode != DQ_P_EQ_NULLSAFE) {
    const bool as_f64 = c[2].arg == DQ_CMP_AS_FLOAT64;
    int col = -1, op = cmp_of(c[2].opcode);
    const PredInsn* lit = nullptr;
    if (numeric_col(c[0]) && lit_ok(c[1])) {
      col = c[0].arg;
      lit = &c[1];
    } else if (lit_ok(c[0]) && numeric_col(c[1])) {
      col = c[1].arg;
      lit = &c[0];
      op = flip_cmp(op);
    }
    if (col < 0) return -1;
    if (!as_f64 && !is_integral(types[col])) return -1;
    fp->kind = FP_CMP;
    fp->op = op;
    fp->as_f64 = as_f64 ? 1 : 0;
    if (!set_lit(*lit, as_f64, &fp->lit_i, &fp->lit_f)) return -1;
    if (as_f64 && fp->lit_f != fp->lit_f) return -1;  // NaN literal: generic path
    return col;
  }
  if (c.size() == 5 && numeric_col(c[0]) && lit_ok(c[1]) && c[2].opcode == DQ_P_COALESCE &&
      lit_ok(c[3]) && cmp_of(c[4].opcode) >= 0 && c[4].opcode != DQ_P_EQ_NULLSAFE) {
    const bool as_f64 = c[4].arg == DQ_CMP_AS_FLOAT64;
    const int col = c[0].arg;
    if (!as_f64 && !is_integral(types[col])) return -1;
    fp->kind = FP_COALESCE_CMP;
    fp->op = cmp_of(c[4].opcode);
    fp->as_f64 = as_f64 ? 1 : 0;
    if (!set_lit(c[3], as_f64, &fp->lit_i, &fp->lit_f)) return -1;
    if (as_f64 && fp->lit_f != fp->lit_f) return -1;  // NaN literal: generic path
    if (!set_lit(c[1], as_f64, &fp->coal_i, &fp->coal_f)) return -1;
    return col;
  }
  return -1;
}

// The specialised 8-byte value scan (dq_scan_fast.hip) runs a task with no `where`, on an
// int64 / fp64 column, with at most one inline `column CMP literal` predicate.  Its compare is
// `x < lit` or `x == lit` (CS_INV negates), so the task's predicate is rewritten here:
// x <= l -> x < l + 1 (int64) / x < nextafter(l, +inf) (fp64).  Returns false (general kernel)
// for every other shape.
static bool fast_variant(ScanTask* t, int* variant) {
  if (t->ptype != DQ_T_INT64 && t->ptype != DQ_T_FLOAT64) return false;
  if (t->n_preds > 1) return false;
  int v = 0;
  if (t->n_preds == 1) {
    FastPred fp = t->preds[0];
    if (fp.kind != FP_CMP) return false;
    const uint32_t cs = fp.cmp_sel & 3u;
    if (cs == CS_MASKS) return false;
    const bool f64 = fp.as_f64 || t->ptype == DQ_T_FLOAT64;
    if (!f64 && t->ptype != DQ_T_INT64) return false;
    if (cs == CS_LE) {
      if (f64) {
        if (!(fp.lit_f < HUGE_VAL)) return false;  // +inf (or NaN): general kernel
        fp.lit_f = std::nextafter(fp.lit_f, HUGE_VAL);
      } else {
        if (fp.lit_i == INT64_MAX) return false;
        fp.lit_i += 1;
      }
      fp.cmp_sel = (fp.cmp_sel & CS_INV) | CS_LT;
    }
    if (f64 && !fp.as_f64) fp.lit_f = (double)fp.lit_i;  // (fp columns: literals are compared as fp)
    const bool lt = (fp.cmp_sel & 3u) == CS_LT;
    v = f64 ? (lt ? 3 : 4) : (lt ? 1 : 2);
    t->preds[0] = fp;
  }
  if (t->flags & TF_STATS) v |= FAST_STATS;
  if (t->flags & TF_HLL) v |= FAST_HLL;
  *variant = v;
  return true;
}

// ------------------------------------------------------------------------------ plan
enum Target { TGT_HOST_SIZE = 0, TGT_SCAN = 1, TGT_HLL = 2, TGT_DTYPE = 3, TGT_STRLEN = 4, TGT_CORR = 5 };

struct OpSlot {
  int kind;
  int target;
  int task;
  int pred;        // COMPLIANCE: predicate slot within the task
  bool has_where;
  int prog_pred = -1;   // generic predicate program evaluating this op's predicate (mask form)
  int prog_where = -1;  // ... and its `where` filter
};

struct TaskBuild {
  int primary;
  int where_prog;  // -1 = none
  ScanTask t;
};

// Scan tasks launched by one kernel specialisation (see launch_scan_group).
struct ScanGroup {
  int kind;   // 0 = validity/mask only, 1 = reads values, 2 = the specialised 8-byte value scan
  int ptype;  // value type (kind 1)
  int np;     // inline predicates (kind 1)
  std::vector<int32_t> tasks;
  size_t dev_offset = 0;  // first entry in d_groups
};

// Per-batch column staging shared by scan plans and frequency tables: host buffers are copied
// (and sliced bitmaps realigned, utf8 offsets rebased -- on the device) into device buffers
// owned here; device buffers are used in place when their layout allows.
//
// Host batches (the JNI path: Arrow buffers in host memory) are double-buffered when the owner
// sets a copy stream: batch k's copies go into staging slot k % 2 on `copy_stream` while the
// kernels of batch k - 1 still run on `stream` (which waits for the copies by event), and a slot
// is refilled only after the kernels that read it two batches ago have finished.
struct Stager {
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // nullptr: copies on `stream` (single slot)
  int slot = 0;                       // staging slot of the batch being prepared
  std::vector<int32_t> col_types;
  std::vector<DevBuf> stage_values[2], stage_validity[2], stage_offsets[2], stage_raw[2];
  std::vector<std::vector<uint8_t>> host_tmp;  // host buffers alive until their copies are done

  void resize_stage(int n_columns) {
    for (int k = 0; k < 2; ++k) {
      stage_values[k].resize(n_columns);
      stage_validity[k].resize(n_columns);
      stage_offsets[k].resize(n_columns);
      stage_raw[k].resize(n_columns);
    }
  }
  hipStream_t copies() const { return copy_stream ? copy_stream : stream; }
};

struct dq_plan : Stager {
  dq_ctx* ctx = nullptr;
  int device = 0;  // of the pooled streams
  std::vector<bool> col_used;
  std::vector<OpSlot> slots;
  std::vector<ScanTask> scan_tasks;
  std::vector<ScanGroup> groups;
  std::vector<int> group_per_cu;  // resident workgroups per CU of each group's kernel (0 = unknown)
  std::vector<HllTask> hll_tasks;    // ApproxCountDistinct not fused into the value scan
  std::vector<std::pair<int, int>> hll_sets;  // (column, where program) of each register set
  std::vector<HllTask> dtype_tasks;  // DataType: {column, type, where, count index}
  // HLL + DataType of the same utf8 (column, where): one fused string pass (dq_string_pass_kernel);
  // the HLL and DataType kernels launch only the tasks not fused here
  std::vector<StrTask> str_tasks;
  std::vector<HllTask> hll_launch, dtype_launch;
  std::vector<HllTask> len_tasks;    // MinLength / MaxLength: {column, type, where}
  std::vector<CorrTask> corr_tasks;  // Correlation: {x, y, where}
  std::vector<Program> programs;  // generic predicate programs -> batch masks
  // device state
  std::vector<dq_status> op_status;  // per op, after dq_plan_finish
  bool pred_cast = false;  // a predicate program casts a string to double (its own kernel: the parser's scratch)
  DevBuf d_tasks, d_groups, d_ranges, d_hll, d_progs, d_insns, d_pool, d_acc, d_partials, d_regs,
      d_cols, d_masks, d_mask_words, d_dtype, d_dtype_counts, d_len, d_len_out, d_corr, d_corr_part, d_corr_acc, d_str;
  int64_t mask_words = 0;
  // pinned descriptor staging (DevColumn + DevMask arrays) guarded by an event
  void* h_desc = nullptr;
  size_t h_desc_size = 0;
  void* h_back = nullptr;  // pinned bounce buffer of dq_plan_finish's readback
  size_t h_back_size = 0;
  hipEvent_t desc_done = nullptr;
  bool desc_pending = false;
  int64_t total_rows = 0;
  int target_blocks = 2048;
  int n_cu = 0;          // compute units of the device (0 = unknown)
  int scan_rounds = 6;   // value-scan grids: whole rounds of resident workgroups (DQ_SCAN_ROUNDS)
  // host batches: staging slot k % 2, filled on copy_stream while the previous batch scans
  uint64_t batch_seq = 0;
  hipEvent_t copy_done[2] = {nullptr, nullptr}, scan_done[2] = {nullptr, nullptr};
  // the fused string pass runs on side_stream beside the value scans of the same batch (both are
  // issue- / latency-bound, so the CUs interleave them); `stream` waits for it before the batch's
  // scan_done, so every later use of the batch's descriptors stays ordered after it
  hipStream_t side_stream = nullptr;
  hipEvent_t side_ready = nullptr, side_done = nullptr;

  ~dq_plan() {
    if (stream) {
      (void)hipStreamSynchronize(stream);
    }
    if (side_stream) (void)hipStreamSynchronize(side_stream);
    if (side_ready) (void)hipEventDestroy(side_ready);
    if (side_done) (void)hipEventDestroy(side_done);
    if (side_stream) StreamPool::get().release(device, side_stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    for (int k = 0; k < 2; ++k) {
      if (copy_done[k]) (void)hipEventDestroy(copy_done[k]);
      if (scan_done[k]) (void)hipEventDestroy(scan_done[k]);
    }
    if (copy_stream) StreamPool::get().release(device, copy_stream);
    if (desc_done) (void)hipEventDestroy(desc_done);
    if (h_desc) PinnedPool::get().release(h_desc);
    if (h_back) PinnedPool::get().release(h_back);
    if (stream) StreamPool::get().release(device, stream);
  }
};

static dq_status check_op(const dq_op& op, const int32_t* types, int n_cols) {
  auto need_col = [&](bool numeric) -> dq_status {
    if (op.column < 0 || op.column >= n_cols) return fail(DQ_ERR_INVALID, "op column out of range");
    if (!valid_type(types[op.column])) return fail(DQ_ERR_INVALID, "invalid column type");
    if (numeric && !is_numeric(types[op.column]))
      return fail(DQ_ERR_UNSUPPORTED, "analyzer needs a numeric column (Preconditions.isNumeric)");
    return DQ_OK;
  };
  switch (op.kind) {
    case DQ_OP_SIZE: break;
    case DQ_OP_COMPLETENESS: DQ_TRY(need_col(false)); break;
    case DQ_OP_COMPLIANCE:
      DQ_TRY(validate_predicate(op.predicate, types, n_cols, nullptr));
      break;
    case DQ_OP_SUM: case DQ_OP_MEAN: case DQ_OP_STDDEV: case DQ_OP_MINIMUM: case DQ_OP_MAXIMUM:
      DQ_TRY(need_col(true));
      break;
    case DQ_OP_APPROX_COUNT_DISTINCT: DQ_TRY(need_col(false)); break;
    case DQ_OP_DATATYPE: DQ_TRY(need_col(false)); break;
    case DQ_OP_MIN_LENGTH: case DQ_OP_MAX_LENGTH:
      DQ_TRY(need_col(false));
      if (types[op.column] != DQ_T_UTF8)
        return fail(DQ_ERR_UNSUPPORTED, "analyzer needs a string column (Preconditions.isString)");
      break;
    case DQ_OP_CORRELATION:
      DQ_TRY(need_col(true));
      if (op.column2 < 0 || op.column2 >= n_cols) return fail(DQ_ERR_INVALID, "op column2 out of range");
      if (!is_numeric(types[op.column2]))
        return fail(DQ_ERR_UNSUPPORTED, "analyzer needs a numeric column (Preconditions.isNumeric)");
      break;
    default: return fail(DQ_ERR_UNSUPPORTED, "unknown op kind " + std::to_string(op.kind));
  }
  if (op.where.code && op.where.n_insns > 0)
    DQ_TRY(validate_predicate(op.where, types, n_cols, nullptr));
  return DQ_OK;
}

extern "C" dq_status dq_op_supported(const dq_op* op, const int32_t* column_types, int n_columns) {
  if (!op || (n_columns > 0 && !column_types)) return fail(DQ_ERR_INVALID, "NULL argument");
  return check_op(*op, column_types, n_columns);
}

static int add_program(dq_plan* plan, Program&& prog) {
  for (size_t i = 0; i < plan->programs.size(); ++i)
    if (plan->programs[i].key == prog.key) return (int)i;
  plan->programs.push_back(std::move(prog));
  return (int)plan->programs.size() - 1;
}

extern "C" dq_status dq_plan_create(dq_ctx* ctx, const dq_op* ops, int n_ops,
                                    const int32_t* column_types, int n_columns, dq_plan** out) {
  if (!out) return fail(DQ_ERR_INVALID, "out is NULL");
  *out = nullptr;
  if (!ctx || (n_ops > 0 && !ops) || n_columns < 0 || (n_columns > 0 && !column_types))
    return fail(DQ_ERR_INVALID, "NULL argument");
  for (int c = 0; c < n_columns; ++c)
    if (!valid_type(column_types[c])) return fail(DQ_ERR_INVALID, "invalid column type");
  for (int i = 0; i < n_ops; ++i) DQ_TRY(check_op(ops[i], column_types, n_columns));

  DQ_HIP(hipSetDevice(ctx->device));
  dq_plan* plan = new dq_plan();
  plan->ctx = ctx;
  plan->col_types.assign(column_types, column_types + n_columns);
  plan->col_used.assign(n_columns, false);

  std::vector<TaskBuild> tasks;
  auto find_or_add_task = [&](int primary, int where_prog) -> int {
    for (size_t i = 0; i < tasks.size(); ++i)
      if (tasks[i].primary == primary && tasks[i].where_prog == where_prog) return (int)i;
    TaskBuild tb;
    tb.primary = primary;
    tb.where_prog = where_prog;
    std::memset(&tb.t, 0, sizeof(tb.t));
    tb.t.primary = primary;
    tb.t.ptype = primary >= 0 ? column_types[primary] : 0;
    tb.t.where_mask = where_prog;
    tb.t.flags = where_prog >= 0 ? TF_WHERE : 0;
    if (primary >= 0) tb.t.flags |= TF_VALIDITY;
    tasks.push_back(tb);
    return (int)tasks.size() - 1;
  };

  dq_status st = DQ_OK;
  for (int i = 0; i < n_ops && st == DQ_OK; ++i) {
    const dq_op& op = ops[i];
    OpSlot slot{op.kind, TGT_SCAN, -1, -1, false};
    int where_prog = -1;
    if (op.where.code && op.where.n_insns > 0) {
      Program wp;
      validate_predicate(op.where, column_types, n_columns, &wp);
      for (int c : wp.columns) plan->col_used[c] = true;
      where_prog = add_program(plan, std::move(wp));
      slot.has_where = true;
      slot.prog_where = where_prog;
    }
    switch (op.kind) {
      case DQ_OP_SIZE: {
        if (where_prog < 0) {
          slot.target = TGT_HOST_SIZE;
        } else {
          int t = -1;  // any task with the same filter can count its rows
          for (size_t k = 0; k < tasks.size(); ++k)
            if (tasks[k].where_prog == where_prog) t = (int)k;
          slot.task = t >= 0 ? t : find_or_add_task(-1, where_prog);
        }
        break;
      }
      case DQ_OP_COMPLETENESS:
        plan->col_used[op.column] = true;
        slot.task = find_or_add_task(op.column, where_prog);
        break;
      case DQ_OP_SUM: case DQ_OP_MEAN: case DQ_OP_STDDEV: case DQ_OP_MINIMUM: case DQ_OP_MAXIMUM: {
        plan->col_used[op.column] = true;
        slot.task = find_or_add_task(op.column, where_prog);
        tasks[slot.task].t.flags |= TF_VALUES | TF_STATS;
        break;
      }
      case DQ_OP_COMPLIANCE: {
        Program pp;
        validate_predicate(op.predicate, column_types, n_columns, &pp);
        for (int c : pp.columns) plan->col_used[c] = true;
        FastPred fp;
        const int fcol = fast_form(pp, column_types, &fp);
        int t;
        if (fcol >= 0) {
          t = find_or_add_task(fcol, where_prog);
          if (fp.kind == FP_CMP || fp.kind == FP_COALESCE_CMP) tasks[t].t.flags |= TF_VALUES;
        } else if (fcol == -2) {
          t = -1;
          for (size_t k = 0; k < tasks.size(); ++k)
            if (tasks[k].where_prog == where_prog) t = (int)k;
          if (t < 0) t = find_or_add_task(-1, where_prog);
        } else {
          const int prog = add_program(plan, std::move(pp));
          fp.kind = FP_MASK;
          fp.mask = prog;
          slot.prog_pred = prog;
          t = -1;  // prefer an existing task with the same filter: masks need no values
          for (size_t k = 0; k < tasks.size(); ++k)
            if (tasks[k].where_prog == where_prog && tasks[k].t.n_preds < kMaxPreds) t = (int)k;
          if (t < 0) t = find_or_add_task(-1, where_prog);
        }
        if (tasks[t].t.n_preds >= kMaxPreds) {
          // task full: open a sibling task on the same column/filter
          TaskBuild tb = tasks[t];
          tb.t.n_preds = 0;
          tb.t.flags &= ~(TF_STATS | TF_HLL);
          tasks.push_back(tb);
          t = (int)tasks.size() - 1;
        }
        slot.task = t;
        slot.pred = tasks[t].t.n_preds;
        finalize_fast_pred(&fp);
        tasks[t].t.preds[tasks[t].t.n_preds++] = fp;
        break;
      }
      case DQ_OP_APPROX_COUNT_DISTINCT: {
        plan->col_used[op.column] = true;
        slot.target = TGT_HLL;
        int t = -1;  // one register set per (column, where)
        for (size_t k = 0; k < plan->hll_sets.size(); ++k)
          if (plan->hll_sets[k] == std::make_pair(op.column, where_prog)) t = (int)k;
        if (t < 0) {
          t = (int)plan->hll_sets.size();
          plan->hll_sets.emplace_back(op.column, where_prog);
          if (is_numeric(column_types[op.column])) {  // hashed in the column's value scan
            const int st_ = find_or_add_task(op.column, where_prog);
            tasks[st_].t.flags |= TF_VALUES | TF_HLL;
            tasks[st_].t.hll = t;
          } else {  // strings / booleans: the HLL kernel
            plan->hll_tasks.push_back(HllTask{op.column, column_types[op.column], where_prog, t});
          }
        }
        slot.task = t;
        break;
      }
      case DQ_OP_DATATYPE: {
        plan->col_used[op.column] = true;
        slot.target = TGT_DTYPE;
        int t = -1;
        for (size_t k = 0; k < plan->dtype_tasks.size(); ++k)
          if (plan->dtype_tasks[k].column == op.column && plan->dtype_tasks[k].where_mask == where_prog)
            t = (int)k;
        if (t < 0) {  // (reg_set = the task's index into the counts: launches may take a subset)
          plan->dtype_tasks.push_back(HllTask{op.column, column_types[op.column], where_prog,
                                              (int32_t)plan->dtype_tasks.size()});
          t = (int)plan->dtype_tasks.size() - 1;
        }
        slot.task = t;
        break;
      }
      case DQ_OP_MIN_LENGTH: case DQ_OP_MAX_LENGTH: {
        plan->col_used[op.column] = true;
        slot.target = TGT_STRLEN;
        int t = -1;
        for (size_t k = 0; k < plan->len_tasks.size(); ++k)
          if (plan->len_tasks[k].column == op.column && plan->len_tasks[k].where_mask == where_prog) t = (int)k;
        if (t < 0) {
          plan->len_tasks.push_back(HllTask{op.column, column_types[op.column], where_prog, 0});
          t = (int)plan->len_tasks.size() - 1;
        }
        slot.task = t;
        break;
      }
      case DQ_OP_CORRELATION: {
        plan->col_used[op.column] = true;
        plan->col_used[op.column2] = true;
        slot.target = TGT_CORR;
        int t = -1;
        for (size_t k = 0; k < plan->corr_tasks.size(); ++k)
          if (plan->corr_tasks[k].x == op.column && plan->corr_tasks[k].y == op.column2 &&
              plan->corr_tasks[k].where_mask == where_prog)
            t = (int)k;
        if (t < 0) {
          plan->corr_tasks.push_back(CorrTask{op.column, op.column2, where_prog, 0});
          t = (int)plan->corr_tasks.size() - 1;
        }
        slot.task = t;
        break;
      }
      default: st = fail(DQ_ERR_UNSUPPORTED, "unknown op kind");
    }
    plan->slots.push_back(slot);
  }
  if (st != DQ_OK) {
    delete plan;
    return st;
  }
  for (auto& tb : tasks) plan->scan_tasks.push_back(tb.t);
  // group tasks by kernel specialisation: (needs values, value type, #inline predicates)
  std::vector<int32_t> group_ids;
  const char* fast_env = std::getenv("DQ_SCAN_FAST");
  const bool fast_on = !(fast_env && fast_env[0] == '0');
  for (size_t i = 0; i < plan->scan_tasks.size(); ++i) {
    ScanTask& t = plan->scan_tasks[i];
    int kind = (t.flags & TF_VALUES) ? 1 : 0;
    const int ptype = kind ? t.ptype : 0;
    bool ext = (t.flags & TF_WHERE) != 0;
    for (int p = 0; p < t.n_preds; ++p) ext = ext || t.preds[p].kind == FP_MASK;
    // np = exact inline-predicate count of a plain task, -1 = the EXT kernel (where/masks)
    int np = kind ? (ext ? -1 : (t.n_preds <= 4 ? t.n_preds : kMaxPreds)) : 0;
    int variant = -1;
    if (fast_on && kind == 1 && !ext && fast_variant(&t, &variant)) {
      kind = 2;  // dq_scan_fast_kernel; np carries the variant
      np = variant;
    }
    ScanGroup* g = nullptr;
    for (auto& gg : plan->groups)
      if (gg.kind == kind && gg.ptype == ptype && gg.np == np) g = &gg;
    if (!g) {
      plan->groups.push_back(ScanGroup{kind, ptype, np, {}, 0});
      g = &plan->groups.back();
    }
    g->tasks.push_back((int32_t)i);
  }
  for (auto& g : plan->groups) {
    g.dev_offset = group_ids.size();
    group_ids.insert(group_ids.end(), g.tasks.begin(), g.tasks.end());
  }

  // device-resident plan tables
  auto upload = [&](DevBuf& buf, const void* src, size_t bytes) -> dq_status {
    if (bytes == 0) return DQ_OK;
    DQ_TRY(buf.ensure(bytes));
    DQ_HIP(hipMemcpy(buf.ptr, src, bytes, hipMemcpyHostToDevice));
    return DQ_OK;
  };
  std::vector<PredProgram> progs;
  std::vector<PredInsn> insns;
  std::string pool;
  plan->pred_cast = false;
  for (const auto& p : plan->programs) {
    progs.push_back(PredProgram{(int32_t)insns.size(), (int32_t)p.code.size()});
    for (PredInsn in : p.code) {
      if (in.opcode == DQ_P_LIT_STRING) in.i64 += (int64_t)pool.size();  // plan-wide pool offset
      if (in.opcode == DQ_P_CAST_DOUBLE) plan->pred_cast = true;
      insns.push_back(in);
    }
    pool += p.pool;
  }
  pool.append(8, '\0');
  // HLL and DataType of the same utf8 (column, where) -- every string column of the profiler's
  // pass 1 -- run as one string pass (one read of the strings); the rest keep their own kernels
  plan->str_tasks.clear();
  plan->hll_launch.clear();
  plan->dtype_launch.clear();
  {
    std::vector<bool> dt_fused(plan->dtype_tasks.size(), false);
    for (const HllTask& h : plan->hll_tasks) {
      int dt = -1;
      if (h.ctype == DQ_T_UTF8 && !getenv_flag("DQ_NO_STRING_PASS"))
        for (size_t k = 0; k < plan->dtype_tasks.size(); ++k)
          if (!dt_fused[k] && plan->dtype_tasks[k].column == h.column && plan->dtype_tasks[k].where_mask == h.where_mask)
            dt = (int)k;
      if (dt >= 0) {
        dt_fused[dt] = true;
        plan->str_tasks.push_back(StrTask{h.column, h.where_mask, h.reg_set, dt});
      } else {
        plan->hll_launch.push_back(h);
      }
    }
    for (size_t k = 0; k < plan->dtype_tasks.size(); ++k)
      if (!dt_fused[k]) plan->dtype_launch.push_back(plan->dtype_tasks[k]);
  }
  dq_status s = DQ_OK;
  if ((s = upload(plan->d_tasks, plan->scan_tasks.data(), plan->scan_tasks.size() * sizeof(ScanTask))) != DQ_OK ||
      (s = upload(plan->d_groups, group_ids.data(), group_ids.size() * sizeof(int32_t))) != DQ_OK ||
      (s = plan->d_ranges.ensure(std::max<size_t>(1, plan->scan_tasks.size()) * sizeof(PartRange))) != DQ_OK ||
      (s = upload(plan->d_hll, plan->hll_launch.data(), plan->hll_launch.size() * sizeof(HllTask))) != DQ_OK ||
      (s = upload(plan->d_dtype, plan->dtype_launch.data(), plan->dtype_launch.size() * sizeof(HllTask))) != DQ_OK ||
      (s = upload(plan->d_str, plan->str_tasks.data(), plan->str_tasks.size() * sizeof(StrTask))) != DQ_OK ||
      (s = plan->d_dtype_counts.ensure(std::max<size_t>(1, plan->dtype_tasks.size()) * 5 * sizeof(uint64_t))) != DQ_OK ||
      (s = upload(plan->d_len, plan->len_tasks.data(), plan->len_tasks.size() * sizeof(HllTask))) != DQ_OK ||
      (s = plan->d_len_out.ensure(std::max<size_t>(1, plan->len_tasks.size()) * 3 * sizeof(uint64_t))) != DQ_OK ||
      (s = upload(plan->d_corr, plan->corr_tasks.data(), plan->corr_tasks.size() * sizeof(CorrTask))) != DQ_OK ||
      (s = plan->d_corr_acc.ensure(std::max<size_t>(1, plan->corr_tasks.size()) * sizeof(CorrAcc))) != DQ_OK ||
      (s = upload(plan->d_progs, progs.data(), progs.size() * sizeof(PredProgram))) != DQ_OK ||
      (s = upload(plan->d_insns, insns.data(), insns.size() * sizeof(PredInsn))) != DQ_OK ||
      (s = upload(plan->d_pool, pool.data(), pool.size())) != DQ_OK ||
      (s = plan->d_acc.ensure(std::max<size_t>(1, plan->scan_tasks.size()) * sizeof(ScanAcc))) != DQ_OK ||
      (s = plan->d_regs.ensure(std::max<size_t>(1, plan->hll_sets.size()) * kHllM * sizeof(uint32_t))) != DQ_OK ||
      (s = plan->d_cols.ensure(std::max(1, n_columns) * sizeof(DevColumn))) != DQ_OK ||
      (s = plan->d_masks.ensure(std::max<size_t>(1, plan->programs.size()) * sizeof(DevMask))) != DQ_OK) {
    delete plan;
    return s;
  }
  plan->device = ctx->device;
  hipError_t e = StreamPool::get().acquire(ctx->device, &plan->stream);
  if (e == hipSuccess) e = StreamPool::get().acquire(ctx->device, &plan->copy_stream);
  for (int k = 0; k < 2 && e == hipSuccess; ++k) {
    e = hipEventCreateWithFlags(&plan->copy_done[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&plan->scan_done[k], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&plan->desc_done, hipEventDisableTiming);
  const char* side_env = std::getenv("DQ_PLAN_SIDE");  // 0: the string pass on the plan's stream (A/B)
  if (e == hipSuccess && !plan->str_tasks.empty() && !(side_env && side_env[0] == '0')) {
    e = StreamPool::get().acquire(ctx->device, &plan->side_stream);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&plan->side_ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&plan->side_done, hipEventDisableTiming);
  }
  plan->h_desc_size = std::max(1, n_columns) * sizeof(DevColumn) +
                      std::max<size_t>(1, plan->programs.size()) * sizeof(DevMask) +
                      std::max<size_t>(1, plan->scan_tasks.size()) * sizeof(PartRange);
  if (e == hipSuccess) e = PinnedPool::get().alloc(plan->h_desc_size, &plan->h_desc);
  if (e != hipSuccess) {
    delete plan;
    return fail(DQ_ERR_DEVICE, std::string("stream/event/pinned allocation failed: ") + hipGetErrorString(e));
  }
  plan->resize_stage(n_columns);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess)
  {
    plan->target_blocks = std::max(256, prop.multiProcessorCount * 8);
    plan->n_cu = prop.multiProcessorCount;
  }
  if (const char* r = std::getenv("DQ_SCAN_ROUNDS")) plan->scan_rounds = std::max(0, std::atoi(r));
  if ((s = dq_plan_reset(plan)) != DQ_OK) {
    delete plan;
    return s;
  }
  *out = plan;
  return DQ_OK;
}

extern "C" dq_status dq_plan_destroy(dq_plan* plan) {
  delete plan;
  return DQ_OK;
}

extern "C" void* dq_plan_stream(dq_plan* plan) { return plan ? (void*)plan->stream : nullptr; }

extern "C" dq_status dq_plan_op_status(dq_plan* plan, int op) {
  if (!plan) return fail(DQ_ERR_INVALID, "plan is NULL");
  if (op < 0 || op >= (int)plan->slots.size()) return fail(DQ_ERR_INVALID, "op index out of range");
  if (plan->op_status.size() != plan->slots.size()) return fail(DQ_ERR_STATE, "dq_plan_finish has not run");
  if (plan->op_status[op] != DQ_OK)
    return fail(plan->op_status[op], "a string -> double cast in this op's predicate met a number off the exact "
                                     "fast path (> 19 significant digits, |exponent| > 22 or hex): route it to Spark");
  return DQ_OK;
}

extern "C" dq_status dq_host_register(void* ptr, size_t bytes) {
  if (!ptr || bytes == 0) return fail(DQ_ERR_INVALID, "NULL or empty host buffer");
  DQ_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
  return DQ_OK;
}

extern "C" dq_status dq_host_unregister(void* ptr) {
  if (!ptr) return fail(DQ_ERR_INVALID, "NULL host buffer");
  DQ_HIP(hipHostUnregister(ptr));
  return DQ_OK;
}

extern "C" dq_status dq_plan_reset(dq_plan* plan) {
  if (!plan) return fail(DQ_ERR_INVALID, "plan is NULL");
  DQ_HIP(hipSetDevice(plan->ctx->device));
  DQ_HIP(launch_init_acc(static_cast<ScanAcc*>(plan->d_acc.ptr), (int)plan->scan_tasks.size(), plan->stream));
  if (!plan->hll_sets.empty())
    DQ_HIP(hipMemsetAsync(plan->d_regs.ptr, 0, plan->hll_sets.size() * kHllM * sizeof(uint32_t), plan->stream));
  if (!plan->dtype_tasks.empty())
    DQ_HIP(hipMemsetAsync(plan->d_dtype_counts.ptr, 0, plan->dtype_tasks.size() * 5 * sizeof(uint64_t), plan->stream));
  if (!plan->len_tasks.empty())
    DQ_HIP(hipMemsetAsync(plan->d_len_out.ptr, 0, plan->len_tasks.size() * 3 * sizeof(uint64_t), plan->stream));
  if (!plan->corr_tasks.empty())  // all-zero CorrAcc = the empty state (n = 0)
    DQ_HIP(hipMemsetAsync(plan->d_corr_acc.ptr, 0, plan->corr_tasks.size() * sizeof(CorrAcc), plan->stream));
  DQ_HIP(hipStreamSynchronize(plan->stream));
  plan->total_rows = 0;
  return DQ_OK;
}

// Host bitmap (bits [off, off + n)) -> LSB-first device bitmap at bit 0: the covering bytes
// are copied as they are and realigned by a kernel on the copy stream (no per-bit host work).
static dq_status stage_host_bitmap(Stager* st, DevBuf& dst, DevBuf& raw, const uint8_t* src, int64_t off,
                                   int64_t n) {
  const size_t vbytes = (size_t)((n + 7) >> 3);
  DQ_TRY(dst.ensure(vbytes + 8));
  if (vbytes == 0) return DQ_OK;
  if ((off & 7) == 0) {
    DQ_HIP(hipMemcpyAsync(dst.ptr, src + (off >> 3), vbytes, hipMemcpyHostToDevice, st->copies()));
    return DQ_OK;
  }
  const size_t first = (size_t)(off >> 3), last = (size_t)((off + n - 1) >> 3);
  DQ_TRY(raw.ensure(last - first + 1 + 8));
  DQ_HIP(hipMemcpyAsync(raw.ptr, src + first, last - first + 1, hipMemcpyHostToDevice, st->copies()));
  DQ_HIP(launch_realign_bitmap(static_cast<const uint8_t*>(raw.ptr), off & 7, n, static_cast<uint8_t*>(dst.ptr),
                               st->copies()));
  return DQ_OK;
}

static dq_status prepare_column(Stager* plan, int c, const dq_column& col, int64_t n_rows,
                                DevColumn* dc) {
  const int t = plan->col_types[c];
  if (col.type != t) return fail(DQ_ERR_INVALID, "column " + std::to_string(c) + " type differs from plan");
  if (col.length < n_rows) return fail(DQ_ERR_INVALID, "column shorter than n_rows");
  if (col.offset < 0) return fail(DQ_ERR_INVALID, "negative column offset");
  if (!col.values && n_rows > 0) return fail(DQ_ERR_INVALID, "column values are NULL");
  if (t == DQ_T_UTF8 && !col.offsets) return fail(DQ_ERR_INVALID, "utf8 column without offsets");
  const bool device = (col.flags & DQ_COL_DEVICE) != 0;
  const int k = plan->slot;
  DevBuf& sval = plan->stage_values[k][c];
  DevBuf& svalid = plan->stage_validity[k][c];
  DevBuf& soffs = plan->stage_offsets[k][c];
  DevBuf& sraw = plan->stage_raw[k][c];
  const int64_t off = col.offset;
  dc->type = t;
  dc->pad = 0;
  dc->offsets = nullptr;
  dc->validity = nullptr;
  const size_t vbytes = (size_t)((n_rows + 7) >> 3);

  // ---- validity
  if (col.validity) {
    if (device) {
      if ((off & 7) == 0) {
        dc->validity = col.validity + (off >> 3);
      } else {
        DQ_TRY(svalid.ensure(vbytes + 8));
        DQ_HIP(launch_realign_bitmap(col.validity, off, n_rows, static_cast<uint8_t*>(svalid.ptr), plan->stream));
        dc->validity = static_cast<const uint8_t*>(svalid.ptr);
      }
    } else {
      DQ_TRY(stage_host_bitmap(plan, svalid, sraw, col.validity, off, n_rows));
      dc->validity = static_cast<const uint8_t*>(svalid.ptr);
    }
  }
  // ---- values
  if (t == DQ_T_BOOL) {
    if (device && (off & 7) == 0) {
      dc->values = static_cast<const uint8_t*>(col.values) + (off >> 3);
    } else if (device) {
      DQ_TRY(sval.ensure(vbytes + 8));
      DQ_HIP(launch_realign_bitmap(static_cast<const uint8_t*>(col.values), off, n_rows,
                                   static_cast<uint8_t*>(sval.ptr), plan->stream));
      dc->values = sval.ptr;
    } else {
      // (the bool bitmap's own raw staging: validity may be using sraw in this slot)
      DevBuf& braw = plan->stage_offsets[k][c];
      DQ_TRY(stage_host_bitmap(plan, sval, braw, static_cast<const uint8_t*>(col.values), off, n_rows));
      dc->values = sval.ptr;
    }
  } else if (t == DQ_T_UTF8) {
    const int32_t* offs = col.offsets + off;
    if (device) {
      dc->offsets = offs;
      dc->values = col.values;
    } else {
      // copy the n + 1 offsets and only the referenced bytes; rebase the offsets on the device
      const int32_t first = n_rows > 0 ? offs[0] : 0;
      const int32_t last = n_rows > 0 ? offs[n_rows] : 0;
      DQ_TRY(soffs.ensure((size_t)(n_rows + 1) * sizeof(int32_t)));
      DQ_TRY(sval.ensure((size_t)(last - first) + 16));
      DQ_HIP(hipMemcpyAsync(soffs.ptr, offs, (size_t)(n_rows + 1) * sizeof(int32_t), hipMemcpyHostToDevice,
                            plan->copies()));
      if (first != 0)
        DQ_HIP(launch_rebase_offsets(static_cast<int32_t*>(soffs.ptr), n_rows + 1, first, plan->copies()));
      if (last > first)
        DQ_HIP(hipMemcpyAsync(sval.ptr, static_cast<const uint8_t*>(col.values) + first, (size_t)(last - first),
                              hipMemcpyHostToDevice, plan->copies()));
      dc->offsets = static_cast<const int32_t*>(soffs.ptr);
      dc->values = sval.ptr;
    }
  } else {
    const size_t es = (size_t)type_size(t);
    const uint8_t* src = static_cast<const uint8_t*>(col.values) + (size_t)off * es;
    const size_t bytes = (size_t)n_rows * es;
    if (device && ((uintptr_t)src & 15) == 0) {
      dc->values = src;
    } else {
      DQ_TRY(sval.ensure(bytes + 16));
      if (bytes)
        DQ_HIP(hipMemcpyAsync(sval.ptr, src, bytes, device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                              device ? plan->stream : plan->copies()));
      dc->values = sval.ptr;
    }
  }
  return DQ_OK;
}

extern "C" dq_status dq_plan_consume(dq_plan* plan, const dq_column* columns, int n_columns,
                                     int64_t n_rows) {
  if (!plan) return fail(DQ_ERR_INVALID, "plan is NULL");
  if (n_columns != (int)plan->col_types.size()) return fail(DQ_ERR_INVALID, "column count differs from plan");
  if (n_rows < 0) return fail(DQ_ERR_INVALID, "negative n_rows");
  if (n_columns > 0 && !columns) return fail(DQ_ERR_INVALID, "columns is NULL");
  if (n_rows == 0) return DQ_OK;
  if (n_rows > (int64_t)1 << 40) return fail(DQ_ERR_INVALID, "batch too large (split it)");
  DQ_HIP(hipSetDevice(plan->ctx->device));

  // the pinned descriptor block may still be in flight from the previous batch
  if (plan->desc_pending) {
    DQ_HIP(hipEventSynchronize(plan->desc_done));
    plan->desc_pending = false;
  }
  DevColumn* h_cols = static_cast<DevColumn*>(plan->h_desc);
  DevMask* h_masks = reinterpret_cast<DevMask*>(static_cast<uint8_t*>(plan->h_desc) +
                                                std::max(1, n_columns) * sizeof(DevColumn));
  bool any_host = false;
  for (int c = 0; c < n_columns; ++c)
    if (plan->col_used[c] && !(columns[c].flags & DQ_COL_DEVICE)) any_host = true;
  const int slot = (int)(plan->batch_seq & 1u);
  plan->slot = slot;
  // this slot's staging was last read by the batch two before: its kernels must have finished
  if (any_host) DQ_HIP(hipStreamWaitEvent(plan->copy_stream, plan->scan_done[slot], 0));
  for (int c = 0; c < n_columns; ++c) {
    std::memset(&h_cols[c], 0, sizeof(DevColumn));
    if (!plan->col_used[c]) continue;
    DQ_TRY(prepare_column(plan, c, columns[c], n_rows, &h_cols[c]));
  }
  if (any_host) {  // the kernels of this batch start once its copies have landed
    DQ_HIP(hipEventRecord(plan->copy_done[slot], plan->copy_stream));
    DQ_HIP(hipStreamWaitEvent(plan->stream, plan->copy_done[slot], 0));
  }
  // generic predicates -> masks
  const int n_progs = (int)plan->programs.size();
  if (n_progs > 0) {
    const int64_t wpm = ((n_rows + 63) >> 6) + 1;
    DQ_TRY(plan->d_mask_words.ensure((size_t)wpm * 2 * n_progs * sizeof(uint64_t)));
    plan->mask_words = wpm;
    uint64_t* base = static_cast<uint64_t*>(plan->d_mask_words.ptr);
    for (int p = 0; p < n_progs; ++p) {
      h_masks[p].t = base + (int64_t)(2 * p) * wpm;
      h_masks[p].nn = base + (int64_t)(2 * p + 1) * wpm;
    }
  }
  // per-group grid sizes and where each task's block partials go for this batch
  const int64_t chunks = (n_rows + kScanRowAlign - 1) / kScanRowAlign;
  const int n_scan = (int)plan->scan_tasks.size();
  PartRange* h_ranges = reinterpret_cast<PartRange*>(reinterpret_cast<uint8_t*>(h_masks) +
                                                     std::max<size_t>(1, plan->programs.size()) * sizeof(DevMask));
  std::vector<int64_t> group_bpt(plan->groups.size()), group_base(plan->groups.size());
  int64_t part_total = 0;
  for (size_t g = 0; g < plan->groups.size(); ++g) {
    const int64_t ng = (int64_t)plan->groups[g].tasks.size();
    int64_t bpt = (plan->target_blocks + ng - 1) / ng;
    const ScanGroup& G = plan->groups[g];
    if (G.kind != 0 && plan->n_cu > 0 && plan->scan_rounds > 0) {
      // the value scans are VALU-bound: one (or scan_rounds) full round(s) of resident
      // workgroups, split evenly over the group's tasks
      if (plan->group_per_cu.size() != plan->groups.size()) {  // once per plan
        plan->group_per_cu.resize(plan->groups.size());
        for (size_t q = 0; q < plan->groups.size(); ++q)
          plan->group_per_cu[q] = plan->groups[q].kind == 0 ? 0
                                  : plan->groups[q].kind == 2
                                      ? scan_fast_blocks_per_cu(plan->groups[q].ptype, plan->groups[q].np)
                                      : scan_group_blocks_per_cu(plan->groups[q].kind, plan->groups[q].ptype,
                                                                 plan->groups[q].np);
      }
      const int per_cu = plan->group_per_cu[g];
      if (per_cu > 0) bpt = std::max<int64_t>(1, (int64_t)plan->n_cu * per_cu * plan->scan_rounds / ng);
    }
    bpt = std::max<int64_t>(1, std::min<int64_t>(bpt, chunks));
    // a block's rows are addressed by 32-bit buffer offsets: keep its span <= 2^27 rows
    bpt = std::max<int64_t>(bpt, (chunks + (((int64_t)1 << 27) / kScanRowAlign) - 1) /
                                     (((int64_t)1 << 27) / kScanRowAlign));
    group_bpt[g] = bpt;
    group_base[g] = part_total;
    for (int64_t i = 0; i < ng; ++i)
      h_ranges[plan->groups[g].tasks[i]] = PartRange{part_total + i * bpt, (int32_t)bpt, 0};
    part_total += bpt * ng;
  }
  if (n_scan > 0) DQ_TRY(plan->d_partials.ensure((size_t)part_total * sizeof(ScanAcc)));

  DQ_HIP(hipMemcpyAsync(plan->d_cols.ptr, h_cols, n_columns * sizeof(DevColumn), hipMemcpyHostToDevice, plan->stream));
  if (n_progs > 0)
    DQ_HIP(hipMemcpyAsync(plan->d_masks.ptr, h_masks, n_progs * sizeof(DevMask), hipMemcpyHostToDevice, plan->stream));
  if (n_scan > 0)
    DQ_HIP(hipMemcpyAsync(plan->d_ranges.ptr, h_ranges, n_scan * sizeof(PartRange), hipMemcpyHostToDevice, plan->stream));
  DQ_HIP(hipEventRecord(plan->desc_done, plan->stream));
  plan->desc_pending = true;

  const DevColumn* d_cols = static_cast<const DevColumn*>(plan->d_cols.ptr);
  const DevMask* d_masks = static_cast<const DevMask*>(plan->d_masks.ptr);
  if (n_progs > 0)
    DQ_HIP(launch_predicates(static_cast<const PredProgram*>(plan->d_progs.ptr), n_progs,
                             static_cast<const PredInsn*>(plan->d_insns.ptr),
                             static_cast<const uint8_t*>(plan->d_pool.ptr), d_cols, n_rows,
                             static_cast<uint64_t*>(plan->d_mask_words.ptr), plan->mask_words, plan->pred_cast,
                             plan->stream));

  const int n_str = (int)plan->str_tasks.size();
  // the string pass first, on the side stream when there is other work to run beside it
  const bool side = n_str > 0 && plan->side_stream && (n_scan > 0 || !plan->hll_launch.empty());
  if (n_str > 0) {
    hipStream_t ss = side ? plan->side_stream : plan->stream;
    if (side) {
      DQ_HIP(hipEventRecord(plan->side_ready, plan->stream));
      DQ_HIP(hipStreamWaitEvent(ss, plan->side_ready, 0));
    }
    int64_t bpt = std::max<int64_t>(1, plan->target_blocks / n_str);
    bpt = std::min<int64_t>(bpt, chunks);
    DQ_HIP(launch_string_pass(static_cast<const StrTask*>(plan->d_str.ptr), n_str, d_cols, d_masks, n_rows, (int)bpt,
                              static_cast<uint32_t*>(plan->d_regs.ptr),
                              static_cast<unsigned long long*>(plan->d_dtype_counts.ptr), ss));
    if (side) DQ_HIP(hipEventRecord(plan->side_done, ss));
  }
  if (n_scan > 0) {
    ScanAcc* parts = static_cast<ScanAcc*>(plan->d_partials.ptr);
    const ScanTask* d_tasks = static_cast<const ScanTask*>(plan->d_tasks.ptr);
    const int32_t* d_groups = static_cast<const int32_t*>(plan->d_groups.ptr);
    for (size_t g = 0; g < plan->groups.size(); ++g) {
      const ScanGroup& G = plan->groups[g];
      if (G.kind == 2)
        DQ_HIP(launch_scan_fast(G.ptype, G.np, d_tasks, d_groups + G.dev_offset, (int)G.tasks.size(), d_cols, n_rows,
                                (int)group_bpt[g], parts + group_base[g], static_cast<uint32_t*>(plan->d_regs.ptr),
                                plan->stream));
      else
        DQ_HIP(launch_scan_group(G.kind, G.ptype, G.np, d_tasks, d_groups + G.dev_offset, (int)G.tasks.size(),
                                 d_cols, d_masks, n_rows, (int)group_bpt[g], parts + group_base[g],
                                 static_cast<uint32_t*>(plan->d_regs.ptr), plan->stream));
    }
    DQ_HIP(launch_scan_reduce(parts, static_cast<const PartRange*>(plan->d_ranges.ptr), n_scan,
                              static_cast<ScanAcc*>(plan->d_acc.ptr), plan->stream));
  }
  const int n_hll = (int)plan->hll_launch.size();
  if (n_hll > 0) {
    int64_t bpt = std::max<int64_t>(1, plan->target_blocks / n_hll);
    bpt = std::min<int64_t>(bpt, chunks);
    DQ_HIP(launch_hll(static_cast<const HllTask*>(plan->d_hll.ptr), n_hll, d_cols, d_masks, n_rows, (int)bpt,
                      static_cast<uint32_t*>(plan->d_regs.ptr), plan->stream));
  }
  const int n_dt = (int)plan->dtype_launch.size();
  if (n_dt > 0) {
    int64_t bpt = std::max<int64_t>(1, plan->target_blocks / n_dt);
    bpt = std::min<int64_t>(bpt, (n_rows + kBlock - 1) / kBlock);
    DQ_HIP(launch_datatype(static_cast<const HllTask*>(plan->d_dtype.ptr), n_dt, d_cols, d_masks, n_rows, (int)bpt,
                           static_cast<unsigned long long*>(plan->d_dtype_counts.ptr), plan->stream));
  }
  const int n_len = (int)plan->len_tasks.size();
  if (n_len > 0) {
    int64_t bpt = std::max<int64_t>(1, plan->target_blocks / n_len);
    bpt = std::min<int64_t>(bpt, (n_rows + kBlock - 1) / kBlock);
    DQ_HIP(launch_strlen(static_cast<const HllTask*>(plan->d_len.ptr), n_len, d_cols, d_masks, n_rows, (int)bpt,
                         static_cast<unsigned long long*>(plan->d_len_out.ptr), plan->stream));
  }
  const int n_corr = (int)plan->corr_tasks.size();
  if (n_corr > 0) {
    int64_t bpt = std::max<int64_t>(1, plan->target_blocks / n_corr);
    bpt = std::min<int64_t>(bpt, (n_rows + kBlock - 1) / kBlock);
    DQ_TRY(plan->d_corr_part.ensure((size_t)n_corr * (size_t)bpt * sizeof(CorrAcc)));
    DQ_HIP(launch_corr(static_cast<const CorrTask*>(plan->d_corr.ptr), n_corr, d_cols, d_masks, n_rows, (int)bpt,
                       static_cast<CorrAcc*>(plan->d_corr_part.ptr), static_cast<CorrAcc*>(plan->d_corr_acc.ptr),
                       plan->stream));
  }
  if (side) DQ_HIP(hipStreamWaitEvent(plan->stream, plan->side_done, 0));
  plan->total_rows += n_rows;
  DQ_HIP(hipEventRecord(plan->scan_done[slot], plan->stream));
  ++plan->batch_seq;
  if (any_host) {  // the caller's host buffers may be released once we return: wait for the
    // copies only -- the scan of this batch keeps running while the caller prepares the next
    DQ_HIP(hipEventSynchronize(plan->copy_done[slot]));
    plan->host_tmp.clear();
  }
  return DQ_OK;
}

static double fsum_value(const ScanAcc& a) {
  if (!std::isfinite(a.fs)) return a.fs;  // Inf/NaN: the plain running sum is Spark's answer
  return a.fs + a.fc;
}

static void pack_hll(const uint32_t* regs, int64_t words[DQ_HLL_NUM_WORDS]) {
  for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) {
    uint64_t word = 0;
    for (int i = 0; i < 10; ++i) {
      const int idx = w * 10 + i;
      if (idx < kHllM) word |= ((uint64_t)(regs[idx] & 63u)) << (6 * i);
    }
    words[w] = (int64_t)word;
  }
}

extern "C" dq_status dq_plan_finish(dq_plan* plan, dq_state* out, int n_out) {
  if (!plan) return fail(DQ_ERR_INVALID, "plan is NULL");
  if (n_out < (int)plan->slots.size() || (!out && !plan->slots.empty()))
    return fail(DQ_ERR_INVALID, "output array too small");
  DQ_HIP(hipSetDevice(plan->ctx->device));
  std::vector<ScanAcc> acc(plan->scan_tasks.size());
  std::vector<uint32_t> regs(plan->hll_sets.size() * kHllM);
  std::vector<uint64_t> dtc(plan->dtype_tasks.size() * 5);
  std::vector<uint64_t> lens(plan->len_tasks.size() * 3);
  std::vector<CorrAcc> corr(plan->corr_tasks.size());
  // every result array comes back in ONE pass through a pinned bounce buffer (pageable copies
  // are staged by the runtime, tens of microseconds each), then one synchronize
  struct Back {
    void* dst;
    const void* src;
    size_t bytes;
  };
  const Back backs[] = {{lens.data(), plan->d_len_out.ptr, lens.size() * sizeof(uint64_t)},
                        {corr.data(), plan->d_corr_acc.ptr, corr.size() * sizeof(CorrAcc)},
                        {dtc.data(), plan->d_dtype_counts.ptr, dtc.size() * sizeof(uint64_t)},
                        {acc.data(), plan->d_acc.ptr, acc.size() * sizeof(ScanAcc)},
                        {regs.data(), plan->d_regs.ptr, regs.size() * sizeof(uint32_t)}};
  size_t total = 0;
  for (const Back& b : backs) total += (b.bytes + 255) & ~(size_t)255;
  if (total > plan->h_back_size) {
    PinnedPool::get().release(plan->h_back);
    plan->h_back = nullptr;
    plan->h_back_size = 0;
    DQ_HIP(PinnedPool::get().alloc(total, &plan->h_back));
    plan->h_back_size = total;
  }
  size_t at = 0;
  for (const Back& b : backs) {
    if (b.bytes)
      DQ_HIP(hipMemcpyAsync(static_cast<uint8_t*>(plan->h_back) + at, b.src, b.bytes, hipMemcpyDeviceToHost,
                            plan->stream));
    at += (b.bytes + 255) & ~(size_t)255;
  }
  DQ_HIP(hipStreamSynchronize(plan->stream));
  at = 0;
  for (const Back& b : backs) {
    if (b.bytes) std::memcpy(b.dst, static_cast<uint8_t*>(plan->h_back) + at, b.bytes);
    at += (b.bytes + 255) & ~(size_t)255;
  }
  plan->op_status.assign(plan->slots.size(), DQ_OK);
  plan->desc_pending = false;
  plan->host_tmp.clear();

  const int64_t rows = plan->total_rows;
  for (size_t i = 0; i < plan->slots.size(); ++i) {
    const OpSlot& s = plan->slots[i];
    dq_state& o = out[i];
    std::memset(&o, 0, sizeof(o));
    o.kind = s.kind;
    if (s.target == TGT_HOST_SIZE) {  // count(*) is never NULL
      o.has_value = 1;
      o.num_matches = rows;
      continue;
    }
    if (s.target == TGT_DTYPE) {  // the StatefulDataType UDAF never returns NULL
      o.has_value = 1;
      for (int k = 0; k < 5; ++k) o.words[k] = (int64_t)dtc[(size_t)s.task * 5 + k];
      continue;
    }
    if (s.target == TGT_STRLEN) {  // min/max(length(...)) is NULL without a selected row
      const uint64_t* l = &lens[(size_t)s.task * 3];
      o.has_value = l[0] > 0;
      o.value = s.kind == DQ_OP_MIN_LENGTH ? (double)(~l[1]) : (double)l[2];
      continue;
    }
    if (s.target == TGT_CORR) {  // Correlation.fromAggregationResult: None unless n > 0 (:85-96)
      const CorrAcc& c = corr[s.task];
      o.has_value = c.n > 0.0;
      o.n = c.n;
      o.avg = c.xavg;
      o.y_avg = c.yavg;
      o.ck = c.ck;
      o.x_mk = c.xmk;
      o.y_mk = c.ymk;
      continue;
    }
    if (s.target == TGT_HLL) {  // never NULL (StatefulHyperloglogPlus.nullable = false)
      o.has_value = 1;
      pack_hll(&regs[(size_t)s.task * kHllM], o.words);
      continue;
    }
    const ScanAcc& a = acc[s.task];
    const int ptype = plan->scan_tasks[s.task].ptype;
    const bool count_ok = s.has_where ? (a.n_wnn > 0) : true;  // conditionalCount non-NULL
    const int64_t count = s.has_where ? a.n_rows : rows;
    switch (s.kind) {
      case DQ_OP_SIZE:
        o.has_value = count_ok ? 1 : 0;
        o.num_matches = count;
        break;
      case DQ_OP_COMPLETENESS:
        o.has_value = (rows > 0 && count_ok) ? 1 : 0;  // sum over zero rows is NULL
        o.num_matches = a.n_sel;
        o.count = count;
        break;
      case DQ_OP_COMPLIANCE:
        o.has_value = (a.pn[s.pred] > 0 && count_ok) ? 1 : 0;
        o.num_matches = a.pm[s.pred];
        o.count = count;
        break;
      case DQ_OP_SUM:
        o.has_value = a.n_sel > 0;
        o.sum = is_integral(ptype) ? (double)a.isum : fsum_value(a);
        break;
      case DQ_OP_MEAN:
        o.has_value = a.n_sel > 0;
        o.sum = is_integral(ptype) ? (double)a.isum : fsum_value(a);
        o.count = a.n_sel;
        break;
      case DQ_OP_STDDEV:
        o.has_value = a.n_sel > 0;
        o.n = (double)a.n_sel;
        o.avg = a.mean;
        o.m2 = a.m2;
        break;
      case DQ_OP_MINIMUM:
        o.has_value = a.n_sel > 0;
        // integral columns: the kernel keeps min/max of (double)x, which equals (double)min(x)
        if (is_integral(ptype)) o.value = a.fmin;
        else o.value = (a.fmin > a.fmax) ? std::numeric_limits<double>::quiet_NaN() : a.fmin;  // all NaN
        break;
      case DQ_OP_MAXIMUM:
        o.has_value = a.n_sel > 0;
        if (is_integral(ptype)) o.value = a.fmax;
        else o.value = a.nnan > 0 ? std::numeric_limits<double>::quiet_NaN() : a.fmax;
        break;
      default: break;
    }
  }
  return DQ_OK;
}

// ------------------------------------------------------------------------------ HLL host
static const double kAlphaM2 = (0.7213 / (1.0 + 1.079 / 512)) * 512.0 * 512.0;

static double estimate_bias(double e) {  // StatefulHyperloglogPlus.scala:259-297
  const double* est = kDqHllRawEstimateP9;
  const int n = DQ_HLL_P9_NUM_ESTIMATES;
  int low = 0, high = n - 1, found = -1;
  while (low <= high) {  // java.util.Arrays.binarySearch(double[], ...)
    const int mid = (low + high) >> 1;
    const double mv = est[mid];
    if (mv < e) low = mid + 1;
    else if (mv > e) high = mid - 1;
    else {
      int64_t mb, kb;
      std::memcpy(&mb, &mv, 8);
      std::memcpy(&kb, &e, 8);
      if (mb == kb) { found = mid; break; }
      if (mb < kb) low = mid + 1;
      else high = mid - 1;
    }
  }
  const int nearest = found >= 0 ? found : low;
  auto dist = [&](int i) { const double d = e - est[i]; return d * d; };
  int lo = std::max(nearest - 6 + 1, 0);
  int hi = std::min(lo + 6, n);
  while (hi < n && dist(hi) < dist(lo)) {
    ++lo;
    ++hi;
  }
  double bias_sum = 0.0;
  for (int i = lo; i < hi; ++i) bias_sum += kDqHllBiasP9[i];
  return bias_sum / (double)(hi - lo);
}

static double java_round(double a) {  // java.lang.Math.round(double) (JDK 8), as a double
  if (std::isnan(a)) return 0.0;
  if (a == 0x1.fffffffffffffp-2) return 0.0;
  const double r = std::floor(a + 0.5);
  if (r >= 9.223372036854775807e18) return 9.223372036854775807e18;
  if (r <= -9.223372036854775808e18) return -9.223372036854775808e18;
  return r;
}

extern "C" double dq_hll_count(const int64_t words[DQ_HLL_NUM_WORDS]) {
  double z_inverse = 0.0, v = 0.0;
  for (int idx = 0; idx < kHllM; ++idx) {
    const uint64_t w = (uint64_t)words[idx / 10];
    const uint32_t m = (uint32_t)((w >> (6 * (idx % 10))) & 63u);
    const int32_t pow2 = (int32_t)(1u << (m & 31u));  // Java int shift of 1 by a Long count
    z_inverse += 1.0 / (double)pow2;
    if (m == 0) v += 1.0;
  }
  auto e_bias_corrected = [&]() {
    const double e = kAlphaM2 / z_inverse;
    return (e < 5.0 * kHllM) ? e - estimate_bias(e) : e;  // P < 19 always holds (P = 9)
  };
  double estimate;
  if (v > 0) {
    const double h = kHllM * std::log((double)kHllM / v);
    estimate = (h <= kDqHllThresholdP9) ? h : e_bias_corrected();
  } else {
    estimate = e_bias_corrected();
  }
  return java_round(estimate);
}

extern "C" void dq_hll_merge(const int64_t a[DQ_HLL_NUM_WORDS], const int64_t b[DQ_HLL_NUM_WORDS],
                             int64_t out[DQ_HLL_NUM_WORDS]) {
  for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) {
    const uint64_t wa = (uint64_t)a[w], wb = (uint64_t)b[w];
    uint64_t word = 0, mask = 63;
    for (int i = 0; i < 10 && w * 10 + i < kHllM; ++i) {
      word |= std::max(wa & mask, wb & mask);
      mask <<= 6;
    }
    out[w] = (int64_t)word;
  }
}

extern "C" void dq_hll_words_to_bytes(const int64_t words[DQ_HLL_NUM_WORDS], uint8_t out[416]) {
  for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w)
    for (int b = 0; b < 8; ++b) out[w * 8 + b] = (uint8_t)((uint64_t)words[w] >> (56 - 8 * b));
}

extern "C" void dq_hll_words_from_bytes(const uint8_t in[416], int64_t words[DQ_HLL_NUM_WORDS]) {
  for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) {
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) v = (v << 8) | in[w * 8 + b];
    words[w] = (int64_t)v;
  }
}

extern "C" uint64_t dq_xxh64(const void* data, size_t len, uint64_t seed) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const uint8_t* end = p + len;
  auto rd64 = [](const uint8_t* q) { uint64_t v; std::memcpy(&v, q, 8); return v; };
  auto rd32 = [](const uint8_t* q) { uint32_t v; std::memcpy(&v, q, 4); return v; };
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
    const uint8_t* limit = end - 32;
    do {
      v1 = xxh_round(v1, rd64(p));
      v2 = xxh_round(v2, rd64(p + 8));
      v3 = xxh_round(v3, rd64(p + 16));
      v4 = xxh_round(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h ^= xxh_round(0, v1); h = h * kP1 + kP4;
    h ^= xxh_round(0, v2); h = h * kP1 + kP4;
    h ^= xxh_round(0, v3); h = h * kP1 + kP4;
    h ^= xxh_round(0, v4); h = h * kP1 + kP4;
  } else {
    h = seed + kP5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xxh_round(0, rd64(p));
    h = rotl64(h, 27) * kP1 + kP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * kP1;
    h = rotl64(h, 23) * kP2 + kP3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * kP5;
    h = rotl64(h, 11) * kP1;
    ++p;
  }
  return xxh_avalanche(h);
}

// ------------------------------------------------------------------------------ state algebra
static double java_min(double a, double b) {  // java.lang.Math.min(double, double)
  if (a != a) return a;
  if (b != b) return b;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? a : b;
  return a <= b ? a : b;
}
static double java_max(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? b : a;
  return a >= b ? a : b;
}

extern "C" dq_status dq_state_merge(const dq_state* a, const dq_state* b, dq_state* out) {
  if (!a || !b || !out) return fail(DQ_ERR_INVALID, "NULL argument");
  if (a->kind != b->kind) return fail(DQ_ERR_INVALID, "cannot merge states of different kinds");
  if (!a->has_value || !b->has_value) {  // Analyzers.merge: None is the identity
    const dq_state* pick = a->has_value ? a : b;
    if (out != pick) *out = *pick;
    return DQ_OK;
  }
  dq_state r = *a;
  switch (a->kind) {
    case DQ_OP_SIZE:  // NumMatches.sum (Size.scala:25-27)
      r.num_matches = (int64_t)((uint64_t)a->num_matches + (uint64_t)b->num_matches);
      break;
    case DQ_OP_COMPLETENESS: case DQ_OP_COMPLIANCE:  // NumMatchesAndCount.sum (Analyzer.scala:233-235)
      r.num_matches = (int64_t)((uint64_t)a->num_matches + (uint64_t)b->num_matches);
      r.count = (int64_t)((uint64_t)a->count + (uint64_t)b->count);
      break;
    case DQ_OP_SUM:  // SumState.sum (Sum.scala:27-29)
      r.sum = a->sum + b->sum;
      break;
    case DQ_OP_MEAN:  // MeanState.sum (Mean.scala:27-29)
      r.sum = a->sum + b->sum;
      r.count = (int64_t)((uint64_t)a->count + (uint64_t)b->count);
      break;
    case DQ_OP_STDDEV: {  // StandardDeviationState.sum (StandardDeviation.scala:37-44)
      const double new_n = a->n + b->n;
      const double delta = b->avg - a->avg;
      const double delta_n = new_n == 0.0 ? 0.0 : delta / new_n;
      r.n = new_n;
      r.avg = a->avg + delta_n * b->n;
      r.m2 = a->m2 + b->m2 + delta * delta_n * a->n * b->n;
      break;
    }
    case DQ_OP_MINIMUM: case DQ_OP_MIN_LENGTH:  // MinState.sum (Minimum.scala:27-29)
      r.value = java_min(a->value, b->value);
      break;
    case DQ_OP_MAXIMUM: case DQ_OP_MAX_LENGTH:  // MaxState.sum (Maximum.scala:27-29)
      r.value = java_max(a->value, b->value);
      break;
    case DQ_OP_CORRELATION: {  // CorrelationState.sum (Correlation.scala:37-52)
      const double n1 = a->n, n2 = b->n, new_n = n1 + n2;
      const double dx = b->avg - a->avg, dx_n = new_n == 0.0 ? 0.0 : dx / new_n;
      const double dy = b->y_avg - a->y_avg, dy_n = new_n == 0.0 ? 0.0 : dy / new_n;
      r.n = new_n;
      r.avg = a->avg + dx_n * n2;
      r.y_avg = a->y_avg + dy_n * n2;
      r.ck = a->ck + b->ck + dx * dy_n * n1 * n2;
      r.x_mk = a->x_mk + b->x_mk + dx * dx_n * n1 * n2;
      r.y_mk = a->y_mk + b->y_mk + dy * dy_n * n1 * n2;
      break;
    }
    case DQ_OP_APPROX_COUNT_DISTINCT: dq_hll_merge(a->words, b->words, r.words); break;
    case DQ_OP_DATATYPE:  // DataTypeHistogram.sum (DataType.scala:48-51)
      for (int k = 0; k < 5; ++k) r.words[k] = (int64_t)((uint64_t)a->words[k] + (uint64_t)b->words[k]);
      break;
    default: return fail(DQ_ERR_INVALID, "unknown state kind");
  }
  *out = r;
  return DQ_OK;
}

extern "C" dq_status dq_state_metric(const dq_state* s, double* out) {
  if (!s || !out) return fail(DQ_ERR_INVALID, "NULL argument");
  if (!s->has_value) return fail(DQ_ERR_STATE, "empty state (all input values were NULL)");
  switch (s->kind) {
    case DQ_OP_SIZE: *out = (double)s->num_matches; break;
    case DQ_OP_COMPLETENESS: case DQ_OP_COMPLIANCE:
      *out = s->count == 0 ? std::numeric_limits<double>::quiet_NaN() : (double)s->num_matches / (double)s->count;
      break;
    case DQ_OP_SUM: *out = s->sum; break;
    case DQ_OP_MEAN:
      *out = s->count == 0 ? std::numeric_limits<double>::quiet_NaN() : s->sum / (double)s->count;
      break;
    case DQ_OP_STDDEV: *out = std::sqrt(s->m2 / s->n); break;
    case DQ_OP_MINIMUM: case DQ_OP_MAXIMUM: case DQ_OP_MIN_LENGTH: case DQ_OP_MAX_LENGTH: *out = s->value; break;
    case DQ_OP_CORRELATION: *out = s->ck / std::sqrt(s->x_mk * s->y_mk); break;  // Correlation.scala:54-56
    case DQ_OP_APPROX_COUNT_DISTINCT: *out = dq_hll_count(s->words); break;
    default: return fail(DQ_ERR_INVALID, "unknown state kind");
  }
  return DQ_OK;
}

// ------------------------------------------------------------------------------ casts
namespace {
struct HostBytes {  // a byte source for the host build of dq_numparse.h
  const uint8_t* p;
  uint32_t operator[](int32_t i) const { return p[i]; }
};
}  // namespace

extern "C" dq_status dq_diag_parse_double(const uint8_t* s, int64_t n, double* out, int32_t* ok) {
  if ((!s && n > 0) || !out || !ok || n < 0 || n > INT32_MAX) return fail(DQ_ERR_INVALID, "bad argument");
  double v = 0.0;
  *ok = numparse::parse_double(HostBytes{s}, (int32_t)n, &v);
  *out = v;
  return DQ_OK;
}

// Host build of the predicate interpreter (dq_predeval.h, the same source dq_pred_kernel runs):
// validates `p` against the columns' types exactly as plan creation does, then evaluates it row
// by row over host columns.  out[r] = 0 FALSE, 1 TRUE, 2 NULL.
extern "C" dq_status dq_diag_eval_predicate(const dq_predicate* p, const dq_column* cols, int n_cols,
                                            int64_t n_rows, uint8_t* out) {
  if (!p || (n_cols > 0 && !cols) || n_cols < 0 || n_rows < 0 || (n_rows > 0 && !out))
    return fail(DQ_ERR_INVALID, "bad argument");
  std::vector<int32_t> types((size_t)n_cols);
  std::vector<DevColumn> dc((size_t)n_cols);
  for (int c = 0; c < n_cols; ++c) {
    if (cols[c].flags & DQ_COL_DEVICE) return fail(DQ_ERR_INVALID, "host columns only");
    if (cols[c].offset != 0) return fail(DQ_ERR_INVALID, "column offset must be 0");
    if (cols[c].length < n_rows) return fail(DQ_ERR_INVALID, "column shorter than n_rows");
    types[c] = cols[c].type;
    dc[c] = DevColumn{cols[c].validity, cols[c].values, cols[c].offsets, cols[c].type, 0};
  }
  Program prog;
  DQ_TRY(validate_predicate(*p, types.data(), n_cols, &prog));
  const uint8_t* pool = reinterpret_cast<const uint8_t*>(prog.pool.data());
  for (int64_t r = 0; r < n_rows; ++r) {
    bool t = false, nn = false;
    pred::eval_program<true>(prog.code.data(), (int)prog.code.size(), pool, dc.data(), r, t, nn);
    out[r] = nn ? (t ? 1 : 0) : 2;
  }
  return DQ_OK;
}

// Host build of the group-by's digit-key packing (dq_keypack.h): the record word of a key of
// <= 15 bytes, and the key bytes it unpacks to.
extern "C" dq_status dq_diag_key_pack(const uint8_t* key, int32_t len, uint64_t* packed, uint8_t* back,
                                      int32_t* back_len, int32_t* ok) {
  if ((!key && len > 0) || !packed || !back || !back_len || !ok || len < 0) return fail(DQ_ERR_INVALID, "bad argument");
  *ok = 0;
  if (len > 15) return DQ_OK;
  uint64_t k[2] = {0, 0};
  std::memcpy(k, key, (size_t)len);
  uint64_t p = 0;
  if (!dq::kp_pack_record(k[0], k[1], (uint32_t)len, &p)) return DQ_OK;
  uint64_t u[2];
  uint32_t n = 0;
  dq::kp_unpack(p, &u[0], &u[1], &n);
  std::memcpy(back, u, n);
  *back_len = (int32_t)n;
  *packed = p;
  *ok = 1;
  return DQ_OK;
}

// Host build of the group-by's UUID packing (dq_uuidpack.h): the two words of a canonical UUID
// key and the 36 text bytes they unpack to.
extern "C" dq_status dq_diag_uuid_pack(const uint8_t* key, int32_t len, uint64_t* words, uint8_t* back, int32_t* ok) {
  if ((!key && len > 0) || !words || !back || !ok || len < 0) return fail(DQ_ERR_INVALID, "bad argument");
  *ok = 0;
  uint64_t lo = 0, hi = 0;
  if (!dq::uuid_pack_bytes(key, (uint32_t)len, &lo, &hi)) return DQ_OK;
  uint32_t w[10];
  dq::uuid_unpack(lo, hi, w);
  std::memcpy(back, w, dq::kUuidLen);
  words[0] = lo;
  words[1] = hi;
  *ok = 1;
  return DQ_OK;
}

extern "C" dq_status dq_cast_utf8(dq_ctx* ctx, const dq_column* src, int64_t n_rows, int32_t to_type,
                                  void* d_values, uint8_t* d_validity, int64_t* n_unsupported) {
  if (!ctx || !src || !n_unsupported || (n_rows > 0 && (!d_values || !d_validity)))
    return fail(DQ_ERR_INVALID, "NULL argument");
  if (src->type != DQ_T_UTF8) return fail(DQ_ERR_INVALID, "dq_cast_utf8 needs a utf8 column");
  if (to_type != DQ_T_INT64 && to_type != DQ_T_FLOAT64) return fail(DQ_ERR_UNSUPPORTED, "cast target must be int64 or float64");
  if (n_rows < 0 || src->length < n_rows) return fail(DQ_ERR_INVALID, "bad n_rows");
  *n_unsupported = 0;
  if (n_rows == 0) return DQ_OK;
  DQ_HIP(hipSetDevice(ctx->device));
  Stager st;
  DQ_HIP(StreamPool::get().acquire(ctx->device, &st.stream));
  st.col_types.assign(1, DQ_T_UTF8);
  st.resize_stage(1);
  DevColumn dc;
  dq_status s = prepare_column(&st, 0, *src, n_rows, &dc);
  hipError_t e = hipSuccess;
  if (s == DQ_OK) e = launch_cast_utf8(dc, n_rows, to_type, d_values, d_validity, st.stream);
  if (s == DQ_OK && e == hipSuccess) e = hipStreamSynchronize(st.stream);
  StreamPool::get().release(ctx->device, st.stream);
  st.stream = nullptr;
  if (s != DQ_OK) return s;
  if (e != hipSuccess) return fail(DQ_ERR_DEVICE, std::string("dq_cast_utf8: ") + hipGetErrorString(e));
  return DQ_OK;
}

// Several columns cast in one call (the profiler's pass 2 casts every string column pass 1 typed
// numeric): the casts alternate over two pooled streams and the call waits once, instead of one
// launch + one synchronisation per column.
extern "C" dq_status dq_cast_utf8_batch(dq_ctx* ctx, int32_t n, const dq_column* srcs, int64_t n_rows,
                                        const int32_t* to_types, void* const* d_values,
                                        uint8_t* const* d_validity) {
  if (!ctx || n < 0 || (n > 0 && (!srcs || !to_types || !d_values || !d_validity)))
    return fail(DQ_ERR_INVALID, "NULL argument");
  for (int32_t i = 0; i < n; ++i) {
    if (srcs[i].type != DQ_T_UTF8) return fail(DQ_ERR_INVALID, "dq_cast_utf8_batch needs utf8 columns");
    if (to_types[i] != DQ_T_INT64 && to_types[i] != DQ_T_FLOAT64)
      return fail(DQ_ERR_UNSUPPORTED, "cast target must be int64 or float64");
    if (n_rows > 0 && (!d_values[i] || !d_validity[i])) return fail(DQ_ERR_INVALID, "NULL output buffer");
  }
  if (n_rows < 0) return fail(DQ_ERR_INVALID, "bad n_rows");
  for (int32_t i = 0; i < n; ++i)
    if (srcs[i].length < n_rows) return fail(DQ_ERR_INVALID, "bad n_rows");
  if (n == 0 || n_rows == 0) return DQ_OK;
  DQ_HIP(hipSetDevice(ctx->device));
  constexpr int kLanes = 2;
  Stager st[kLanes];
  dq_status s = DQ_OK;
  hipError_t e = hipSuccess;
  int acquired = 0;
  for (; acquired < kLanes && e == hipSuccess; ++acquired) {
    e = StreamPool::get().acquire(ctx->device, &st[acquired].stream);
    if (e != hipSuccess) break;
    st[acquired].col_types.assign((size_t)n, DQ_T_UTF8);
    st[acquired].resize_stage(n);
  }
  for (int32_t i = 0; i < n && e == hipSuccess && s == DQ_OK; ++i) {
    Stager& L = st[i % kLanes];
    DevColumn dc;
    s = prepare_column(&L, i, srcs[i], n_rows, &dc);
    if (s == DQ_OK) e = launch_cast_utf8(dc, n_rows, to_types[i], d_values[i], d_validity[i], L.stream);
  }
  for (int k = 0; k < acquired; ++k) {
    const hipError_t w = hipStreamSynchronize(st[k].stream);
    if (e == hipSuccess) e = w;
    StreamPool::get().release(ctx->device, st[k].stream);
    st[k].stream = nullptr;
  }
  if (s != DQ_OK) return s;
  if (e != hipSuccess) return fail(DQ_ERR_DEVICE, std::string("dq_cast_utf8_batch: ") + hipGetErrorString(e));
  return DQ_OK;
}

extern "C" dq_status dq_profile_string_groups(dq_ctx* ctx, const int64_t* counts, const int64_t* key_offsets,
                                              const uint8_t* key_bytes, int64_t n_groups, int64_t n_nulls, int flags,
                                              dq_state* hll_out, dq_state* dtype_out) {
  if (!ctx || !hll_out || !dtype_out || n_groups < 0 || n_nulls < 0 || (n_groups > 0 && (!counts || !key_offsets)))
    return fail(DQ_ERR_INVALID, "bad argument");
  if (flags & ~DQ_FLAT_DEVICE) return fail(DQ_ERR_INVALID, "unknown flag");
  const bool dev = (flags & DQ_FLAT_DEVICE) != 0;
  DQ_HIP(hipSetDevice(ctx->device));
  hipStream_t stream = nullptr;
  DQ_HIP(StreamPool::get().acquire(ctx->device, &stream));
  struct Release {
    int d;
    hipStream_t s;
    ~Release() { StreamPool::get().release(d, s); }
  } rel{ctx->device, stream};
  int64_t n_bytes = 0;
  if (n_groups > 0) {
    if (dev)
      DQ_HIP(hipMemcpyAsync(&n_bytes, key_offsets + n_groups, 8, hipMemcpyDeviceToHost, stream));
    else
      n_bytes = key_offsets[n_groups];
    DQ_HIP(hipStreamSynchronize(stream));
    if (n_bytes < 0 || (n_bytes > 0 && !key_bytes)) return fail(DQ_ERR_INVALID, "bad key bytes");
  }
  const size_t a = (size_t)n_groups * 8, b = ((size_t)n_groups + 1) * 8, c = (size_t)n_bytes;
  const size_t scratch = kHllM * sizeof(uint32_t) + 8 * sizeof(unsigned long long);
  DevBuf buf;
  DQ_TRY(buf.ensure(scratch + (dev ? 0 : a + b + c + 16)));
  uint8_t* base = static_cast<uint8_t*>(buf.ptr);
  uint32_t* d_regs = reinterpret_cast<uint32_t*>(base);
  unsigned long long* d_dtc = reinterpret_cast<unsigned long long*>(base + kHllM * sizeof(uint32_t));
  DQ_HIP(hipMemsetAsync(base, 0, scratch, stream));
  const int64_t* d_cnt = counts;
  const int64_t* d_off = key_offsets;
  const uint8_t* d_bytes = key_bytes;
  if (!dev && n_groups > 0) {
    uint8_t* in = base + scratch;
    DQ_HIP(hipMemcpyAsync(in, counts, a, hipMemcpyHostToDevice, stream));
    DQ_HIP(hipMemcpyAsync(in + a, key_offsets, b, hipMemcpyHostToDevice, stream));
    if (c) DQ_HIP(hipMemcpyAsync(in + a + b, key_bytes, c, hipMemcpyHostToDevice, stream));
    d_cnt = reinterpret_cast<const int64_t*>(in);
    d_off = reinterpret_cast<const int64_t*>(in + a);
    d_bytes = in + a + b;
  }
  DQ_HIP(launch_string_groups(d_cnt, d_off, d_bytes, n_groups, d_regs, d_dtc, stream));
  std::vector<uint32_t> regs(kHllM);
  unsigned long long dtc[5];
  DQ_HIP(hipMemcpyAsync(regs.data(), d_regs, kHllM * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  DQ_HIP(hipMemcpyAsync(dtc, d_dtc, sizeof(dtc), hipMemcpyDeviceToHost, stream));
  DQ_HIP(hipStreamSynchronize(stream));
  std::memset(hll_out, 0, sizeof(*hll_out));
  hll_out->kind = DQ_OP_APPROX_COUNT_DISTINCT;
  hll_out->has_value = 1;  // never NULL (StatefulHyperloglogPlus.nullable = false)
  pack_hll(regs.data(), hll_out->words);
  std::memset(dtype_out, 0, sizeof(*dtype_out));
  dtype_out->kind = DQ_OP_DATATYPE;
  dtype_out->has_value = 1;  // the StatefulDataType UDAF never returns NULL
  for (int k = 0; k < 5; ++k) dtype_out->words[k] = (int64_t)dtc[k];
  dtype_out->words[0] += n_nulls;  // (DtPos: NULL first, dq_profile.hip)
  return DQ_OK;
}

// One chunk of dq_profile_few_strings' columns (arguments checked, results zeroed by the caller).
static dq_status few_strings_chunk(dq_ctx* ctx, int32_t n, const dq_column* cols, int64_t n_rows,
                                   dq_few_result* results, int64_t* group_counts, uint8_t* group_keys,
                                   int32_t* group_lens) {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
  // every column in ONE launch of each kernel (blockIdx.y = column): the few-groups kernel (its
  // workgroups' lists), the per-column merge into one compact list, the states from the groups
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(2 * (int64_t)cus, n_rows / 4096));
  const size_t nc = (size_t)n, per = (size_t)blocks * kFreqSmallSlots, S = kFreqSmallSlots;
  const size_t lists = nc * per * (8 + 8 + 4) + nc * (size_t)blocks * 4;
  const size_t outs_bytes = nc * S * 24 + nc * 8 + nc * kHllM * sizeof(uint32_t) + nc * 8 * sizeof(unsigned long long);
  DevBuf scratch, outs, dcols;
  DQ_TRY(scratch.ensure(lists));
  DQ_TRY(outs.ensure(outs_bytes));
  DQ_TRY(dcols.ensure(sizeof(DevColumn) * nc));
  Stager st;
  DQ_HIP(StreamPool::get().acquire(ctx->device, &st.stream));
  struct Release {
    int d;
    Stager* s;
    ~Release() { StreamPool::get().release(d, s->stream); s->stream = nullptr; }
  } rel{ctx->device, &st};
  st.col_types.assign(nc, DQ_T_UTF8);
  st.resize_stage(n);
  std::vector<DevColumn> hc(nc);
  for (int32_t i = 0; i < n; ++i) DQ_TRY(prepare_column(&st, i, cols[i], n_rows, &hc[(size_t)i]));
  DQ_HIP(hipMemcpyAsync(dcols.ptr, hc.data(), sizeof(DevColumn) * nc, hipMemcpyHostToDevice, st.stream));
  uint8_t* lb = static_cast<uint8_t*>(scratch.ptr);
  unsigned long long* k0 = reinterpret_cast<unsigned long long*>(lb);
  unsigned long long* k1 = k0 + nc * per;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(k1 + nc * per);
  uint32_t* nused = cnt + nc * per;
  uint8_t* ob = static_cast<uint8_t*>(outs.ptr);
  unsigned long long* ok0 = reinterpret_cast<unsigned long long*>(ob);
  unsigned long long* ok1 = ok0 + nc * S;
  unsigned long long* oc = ok1 + nc * S;
  uint32_t* on = reinterpret_cast<uint32_t*>(oc + nc * S);
  unsigned int* bad = on + nc;
  uint32_t* regs = bad + nc;
  unsigned long long* dtc = reinterpret_cast<unsigned long long*>(regs + nc * kHllM);
  DQ_HIP(hipMemsetAsync(on, 0, nc * 8 + nc * kHllM * sizeof(uint32_t) + nc * 8 * sizeof(unsigned long long), st.stream));
  FreqKeySpec ks{};
  ks.key_cols[0] = 0;
  ks.n_keys = 1;
  ks.null_as_key = 0;
  DQ_HIP(launch_freq_small_flat(true, ks, static_cast<const DevColumn*>(dcols.ptr), n, n_rows, blocks, k0, k1, cnt, nused,
                                bad, ok0, ok1, oc, on, st.stream));
  DQ_HIP(launch_string_groups_words(ok0, ok1, oc, on, kFreqSmallSlots, n, regs, dtc, st.stream));
  std::vector<uint8_t> host(outs_bytes);
  DQ_HIP(hipMemcpyAsync(host.data(), ob, outs_bytes, hipMemcpyDeviceToHost, st.stream));
  DQ_HIP(hipStreamSynchronize(st.stream));
  const unsigned long long* hk0 = reinterpret_cast<const unsigned long long*>(host.data());
  const unsigned long long* hk1 = hk0 + nc * S;
  const unsigned long long* hcn = hk1 + nc * S;
  const uint32_t* hn = reinterpret_cast<const uint32_t*>(hcn + nc * S);
  const uint32_t* hbad = hn + nc;
  const uint32_t* hregs = hbad + nc;
  const unsigned long long* hdtc = reinterpret_cast<const unsigned long long*>(hregs + nc * kHllM);
  for (int32_t i = 0; i < n; ++i) {
    if (hbad[i]) continue;  // (more groups, a longer key, or a heap under 16 bytes: the per-row pass)
    dq_few_result& r = results[i];
    const uint32_t ng = hn[i];
    uint64_t grouped = 0;
    for (uint32_t g = 0; g < ng; ++g) {
      const size_t at = (size_t)i * S + g;
      group_counts[at] = (int64_t)hcn[at];
      group_lens[at] = (int32_t)(hk1[at] >> 56);
      for (int b = 0; b < 8; ++b) group_keys[at * 16 + b] = (uint8_t)(hk0[at] >> (8 * b));
      for (int b = 0; b < 8; ++b) group_keys[at * 16 + 8 + b] = b < 7 ? (uint8_t)(hk1[at] >> (8 * b)) : 0;
      grouped += hcn[at];
    }
    r.ok = 1;
    r.n_groups = (int32_t)ng;
    r.n_nulls = n_rows - (int64_t)grouped;
    r.completeness.kind = DQ_OP_COMPLETENESS;
    r.completeness.has_value = 1;  // (n_rows > 0)
    r.completeness.num_matches = (int64_t)grouped;
    r.completeness.count = n_rows;
    r.hll.kind = DQ_OP_APPROX_COUNT_DISTINCT;
    r.hll.has_value = 1;
    pack_hll(hregs + (size_t)i * kHllM, r.hll.words);
    r.dtype.kind = DQ_OP_DATATYPE;
    r.dtype.has_value = 1;
    for (int k = 0; k < 5; ++k) r.dtype.words[k] = (int64_t)hdtc[(size_t)i * 8 + k];
    r.dtype.words[0] += r.n_nulls;  // (DtPos: NULL first, dq_profile.hip)
  }
  return DQ_OK;
}

extern "C" dq_status dq_profile_few_strings(dq_ctx* ctx, int32_t n, const dq_column* cols, int64_t n_rows,
                                            dq_few_result* results, int64_t* group_counts, uint8_t* group_keys,
                                            int32_t* group_lens) {
  static_assert(DQ_FEW_MAX_GROUPS == kFreqSmallSlots, "the few-groups kernel's LDS table size");
  if (!ctx || n < 0 || (n > 0 && (!cols || !results || !group_counts || !group_keys || !group_lens)))
    return fail(DQ_ERR_INVALID, "NULL argument");
  if (n_rows < 0 || n > 65535) return fail(DQ_ERR_INVALID, "bad n_rows or column count");
  for (int32_t i = 0; i < n; ++i) {
    if (cols[i].type != DQ_T_UTF8) return fail(DQ_ERR_INVALID, "dq_profile_few_strings needs utf8 columns");
    if (cols[i].length < n_rows) return fail(DQ_ERR_INVALID, "bad n_rows");
  }
  std::memset(results, 0, sizeof(dq_few_result) * (size_t)std::max(0, n));
  if (n == 0 || n_rows == 0) return DQ_OK;  // (no rows: every column goes to the per-row pass)
  DQ_HIP(hipSetDevice(ctx->device));
  // Bounded chunks: the workgroup lists take blocks x 1024 x 20 B per column (~12 MB on 304
  // CUs), so a wide table is grouped 32 columns at a time.  A chunk whose scratch cannot be
  // allocated is not an error: its columns stay ok = 0 and take the per-row string pass.
  constexpr int32_t kChunk = 32;
  const size_t S = kFreqSmallSlots;
  for (int32_t i0 = 0; i0 < n; i0 += kChunk) {
    const int32_t m = std::min(kChunk, n - i0);
    const dq_status st = few_strings_chunk(ctx, m, cols + i0, n_rows, results + i0, group_counts + (size_t)i0 * S,
                                           group_keys + (size_t)i0 * S * 16, group_lens + (size_t)i0 * S);
    if (st == DQ_ERR_OOM) {
      (void)hipGetLastError();  // (clear the runtime's sticky allocation error)
      std::memset(results + i0, 0, sizeof(dq_few_result) * (size_t)m);
      continue;
    }
    if (st != DQ_OK) return st;
  }
  return DQ_OK;
}

// The frequency group-by shares the staging helpers above.
#include "dq_freq_api.inc"

// Arrow C Data Interface entry points over dq_plan_consume / dq_freq_consume.
#include "dq_arrow.inc"

// RCCL groups: the sharded path's collectives for drivers that are not torch.
#include "dq_group.inc"

// The analyzer list as the JVM serializes it.
#include "dq_packed.inc"
