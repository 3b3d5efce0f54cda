// backend.hip -- context, device memory, keys, CKKS operators and the
// Lattigo-compatible C-ABI of liborion_hip.so (include/orion_hip.h).
//
// Operator algorithms follow Lattigo v6 as reached from
// /root/reference/orion/backend/lattigo/*.go; the CPU
// restatement they are checked against lives in oracle/ (tests only).
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>
#include <complex>

#include "../../include/orion_hip.h"
#include "common.h"
#include "hostmath.h"
#include "wire.h"

int orion_launch_ntt(int logN, const LimbSet& s, const DeviceTables* tb, bool inverse, hipStream_t st);
int orion_launch_ntt_io(int logN, const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st);
int orion_launch_ntt2(int logN, const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st);
int orion_launch_ntt2s(int logN, const NttIO& io, const DeviceTables* tb, bool inverse, hipStream_t st,
                       bool rows_only = false);
int orion_ntt_init();
int orion_launch_ew(int op, const LimbSet& o, const LimbSet& a, const LimbSet& b, const u64* s, const u64* ss,
                    const DeviceTables* tb, int N, hipStream_t st);
int orion_launch_tensor(const LimbSet& d, const LimbSet& a, const LimbSet& b, const DeviceTables* tb, int N,
                        hipStream_t st);
int orion_launch_basis_ext(const LimbSet& out, const LimbSet& in, const BasisExtTable* T, const DeviceTables* tb,
                           int N, hipStream_t st);
int orion_launch_modup_all(const LimbSet& D, const LimbSet& in, const BasisExtTable* Ts, int beta, int K,
                           int nqp, const DeviceTables* tb, int N, hipStream_t st);
int orion_launch_ks_mac(const LimbSet& out, const LimbSet& D, const LimbSet& own, const MacGroups& G, int ngroup,
                        int beta, const DeviceTables* tb, int N, hipStream_t st);
int orion_launch_automorph(const LimbSet& o, const LimbSet& a, const u32* idx, const DeviceTables* tb, int N,
                           int accumulate, hipStream_t st);
int orion_launch_lt_bsgs(const LimbSet& t0, const LimbSet& t1, const LimbSet& D, const LimbSet& ct,
                         const LtBabies& Bb, const LtPlan* plan, int g0, int g1, int accumulate, const LimbSet& ptl,
                         const DeviceTables* tb, int N, hipStream_t st);
int orion_launch_lt_giant(const LimbSet& acc, const LimbSet& D, const LimbSet& own, const LimbSet& t0,
                          const LimbSet& z, const LtGiants& G, const DeviceTables* tb, int N, hipStream_t st);

int orion_launch_encode(const float* vals, int nvals, int B, double2* v, const double2* tw_inv, int logn, bool ci,
                        const LimbSet& out, double scale, const DeviceTables* tb, hipStream_t st);
int orion_launch_decode(const LimbSet& x, const u64* garner, double scale, int logn, bool ci, double2* v,
                        const double2* tw_fwd, double* out, const DeviceTables* tb, hipStream_t st);
int orion_launch_enc_sample(const LimbSet& r, const EncSampler& sp, const DeviceTables* tb, int N, hipStream_t st);
int orion_launch_encode_c(double2* v, int B, const double2* tw_inv, int logn, bool ci, const LimbSet& out, double scale,
                          const DeviceTables* tb, hipStream_t st);
int orion_launch_modraise(const LimbSet& out, const LimbSet& in, const DeviceTables* tb, int N, hipStream_t st);

static void bsgs_split(int rot, int slots, int N1, int* giant, int* baby);
static int find_best_n1(const std::vector<int>& idx, int slots, int logMaxRatio);

namespace orion {

enum { EW_ADD = 0, EW_SUB, EW_MUL, EW_MULADD, EW_NEG, EW_SCALE, EW_ADDC, EW_SUBSCALE, EW_COPY, EW_ADDSCALE, EW_SPLIT24 };

#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + \
                                                   " at " + #x);                                   \
  } while (0)

static thread_local std::string g_last_error;

// ---------------------------------------------------------------------------
// device memory: size-class cache (no hipMalloc/hipFree on the op path)
// ---------------------------------------------------------------------------
// A captured hipGraph replays into the buffers its capture used, so every
// buffer handed out while capturing is pinned for the graph's lifetime: a
// pinned buffer that is released is parked instead of returning to the free
// lists, and nothing allocated later can alias a graph's temporaries.
class DevicePool {
  // ORION_DEBUG_POISON=1: fill each allocation with 0xA5 bytes, so a kernel that
  // reads memory nothing wrote fails deterministically
  bool poison_ = getenv("ORION_DEBUG_POISON") && atoi(getenv("ORION_DEBUG_POISON")) != 0;

 public:
  // every pool of the process shares one lock: the pipelines' contexts run on
  // threads of their own, a forced trim empties every pool, and a buffer can be
  // released by another context's thread than the one that allocated it (keys
  // and compiled objects are shared with the pipelines)
  static std::recursive_mutex& mu() {
    static auto* m = new std::recursive_mutex();
    return *m;
  }
  // ORION_POOL_CAP_BYTES: the device bytes all pools together may hold; an
  // allocation past it takes the failed-hipMalloc path (trim every pool's
  // cache, retry once) -- the regression test of that path, and a way to run
  // a workload inside a memory budget
  static double& cap_ref() {
    static double c = getenv("ORION_POOL_CAP_BYTES") ? atof(getenv("ORION_POOL_CAP_BYTES")) : 0;
    return c;
  }
  static double cap_bytes() { return cap_ref(); }
  // A cached buffer is reused for a request of up to its size when the
  // request is at least 7/8 of it (best fit): the limb counts of a chain's
  // levels make many nearby sizes, and exact-size classes alone left memory
  // cached in sizes no request took (ResNet-20 N=2^16 at batch 8 thrashed).
  void* alloc(size_t bytes) {
    std::lock_guard<std::recursive_mutex> lk(mu());
    void* p = nullptr;
    auto it = free_.lower_bound(bytes);
    if (it != free_.end() && it->first - bytes <= it->first / 8) {
      p = it->second.back();
      it->second.pop_back();
      if (it->second.empty()) free_.erase(it);
    } else {
      const bool over = cap_bytes() > 0 && stats()[0] + (double)bytes > cap_bytes();
      hipError_t e = over ? hipErrorOutOfMemory : hipMalloc(&p, bytes);
      if (e != hipSuccess) {
        // release cached buffers of every pool on the device (the scheme's,
        // its pipelines' and the bootstrappers' contexts), the largest first,
        // until the request fits; then, if it still does not, every cache --
        // not while capturing: a trim synchronises.  The failed call's error
        // is cleared: HIP keeps it as the thread's last error, and a later
        // launch check (hipGetLastError) would report it
        (void)hipGetLastError();
        for (DevicePool* q : registry())
          if (q->tracking_) throw std::runtime_error("device memory exhausted during graph capture");
        stats()[3] += 1;  // one forced trim per failed allocation, whatever the number of pools
        // first, the smallest cached buffer of any pool that is large enough
        // is taken over as it is (no free, no allocation: under memory
        // pressure a larger buffer serves the request); the device is drained
        // first, since another context's stream may still use its cache
        hipDeviceSynchronize();
        p = adopt_cached(bytes);
        if (p) {
          if (tracking_) touched_[p] = bytes;
          return p;
        }
        for (int pass = 0; pass < 2; ++pass) {
          // pass 0: twice the request (at least 1 GiB) from the largest
          // cached buffers; pass 1: everything
          trim_largest(pass == 0 ? std::max<size_t>(2 * bytes, (size_t)1 << 30) : SIZE_MAX);
          if (cap_bytes() > 0 && stats()[0] + (double)bytes > cap_bytes()) {
            if (pass == 0) continue;
            throw std::runtime_error("device memory exhausted: " + std::to_string(bytes) +
                                     " more bytes exceed the pool cap (ORION_POOL_CAP_BYTES) with every cache released");
          }
          e = hipMalloc(&p, bytes);
          if (e == hipSuccess) break;
          (void)hipGetLastError();
          if (pass == 1)
            throw std::runtime_error("device memory exhausted: hipMalloc of " + std::to_string(bytes) +
                                     " bytes failed with every pool's cache released (" +
                                     std::to_string((long long)stats()[0]) + " bytes held by live objects)");
        }
      }
      stats()[2] += 1;
      held_ += bytes;
      real_[p] = bytes;
      add_held((double)bytes);
    }
    if (tracking_) touched_[p] = bytes;
    // debugging: every buffer handed out holds garbage, not stale or zero pages
    // (skipped inside a graph capture: a device sync there would invalidate it)
    if (poison_ && !tracking_) {
      (void)hipDeviceSynchronize();
      (void)hipMemset(p, 0xA5, bytes);
    }
    return p;
  }
  // a pointer's allocated size (>= the bytes its holder asked for)
  size_t real(void* p) const {
    auto it = real_.find(p);
    return it == real_.end() ? 0 : it->second;
  }
  void release(void* p, size_t bytes) {
    std::lock_guard<std::recursive_mutex> lk(mu());
    bytes = real(p);  // cached by its allocated size
    if (pins_.count(p)) {
      parked_[p] = bytes;
      return;
    }
    if (tracking_ && !touched_.count(p)) {
      // predates the open capture: the captured work may read it at every
      // replay, so nothing recorded later in the capture may reuse it; it is
      // parked now and pinned with the graph's buffers at the end
      touched_[p] = bytes;
      parked_[p] = bytes;
      return;
    }
    free_[bytes].push_back(p);
  }
  // a capture that failed: buffers parked for it that no graph pins go back
  void unpark_unpinned(const std::vector<std::pair<void*, size_t>>& v) {
    std::lock_guard<std::recursive_mutex> lk(mu());
    for (auto& pb : v) {
      if (pins_.count(pb.first)) continue;
      auto pk = parked_.find(pb.first);
      if (pk != parked_.end()) {
        free_[real(pk->first)].push_back(pk->first);
        parked_.erase(pk);
      }
    }
  }
  // free the cached (unused) buffers
  void trim() {
    std::lock_guard<std::recursive_mutex> lk(mu());
    hipDeviceSynchronize();
    for (auto& kv : free_)
      for (void* p : kv.second) free_one(p);
    free_.clear();
  }
  // the smallest cached buffer of at least `bytes` in any pool, moved into
  // this pool (nullptr: none); the caller has drained the device
  void* adopt_cached(size_t bytes) {
    DevicePool* best = nullptr;
    size_t bsz = SIZE_MAX;
    for (DevicePool* q : registry()) {
      auto it = q->free_.lower_bound(bytes);
      if (it != q->free_.end() && it->first < bsz) best = q, bsz = it->first;
    }
    if (!best) return nullptr;
    auto it = best->free_.find(bsz);
    void* p = it->second.back();
    it->second.pop_back();
    if (it->second.empty()) best->free_.erase(it);
    if (best != this) {
      best->real_.erase(p);
      best->held_ -= bsz;
      real_[p] = bsz;
      held_ += bsz;
    }
    return p;
  }
  // free cached buffers of every pool, the largest first, until `need` bytes
  // are freed (or every cache is empty)
  static void trim_largest(size_t need) {
    std::lock_guard<std::recursive_mutex> lk(mu());
    hipDeviceSynchronize();
    std::vector<std::pair<size_t, DevicePool*>> sizes;
    for (DevicePool* q : registry())
      for (auto& kv : q->free_)
        if (!kv.second.empty()) sizes.push_back({kv.first, q});
    std::sort(sizes.begin(), sizes.end(), [](const std::pair<size_t, DevicePool*>& x,
                                              const std::pair<size_t, DevicePool*>& y) { return x.first > y.first; });
    size_t freed = 0;
    for (auto& sq : sizes) {
      auto it = sq.second->free_.find(sq.first);
      while (freed < need && it != sq.second->free_.end() && !it->second.empty()) {
        sq.second->free_one(it->second.back());
        it->second.pop_back();
        freed += sq.first;
      }
      if (it != sq.second->free_.end() && it->second.empty()) sq.second->free_.erase(it);
      if (freed >= need) break;
    }
  }
  DevicePool() {
    std::lock_guard<std::recursive_mutex> lk(mu());
    registry().push_back(this);
  }
  DevicePool(const DevicePool&) = delete;
  DevicePool& operator=(const DevicePool&) = delete;
  // every pool of the process (one per context), and process-wide counters:
  // device bytes held by the pools (handed out + cached), their peak,
  // hipMalloc calls, failed allocations that forced a trim of every cache
  static std::vector<DevicePool*>& registry() {
    // never destroyed: contexts held in namespace-scope statics are torn down
    // at library unload, possibly after a function-local static would be
    static auto* r = new std::vector<DevicePool*>();
    return *r;
  }
  static double* stats() {
    static double st[4] = {0, 0, 0, 0};
    return st;
  }
  static void add_held(double d) {
    stats()[0] += d;
    if (stats()[0] > stats()[1]) stats()[1] = stats()[0];
  }
  size_t cached() const {
    std::lock_guard<std::recursive_mutex> lk(mu());
    size_t c = 0;
    for (auto& kv : free_) c += kv.first * kv.second.size();
    return c;
  }
  // graph capture: record every buffer handed out until end_track()
  void begin_track() {
    std::lock_guard<std::recursive_mutex> lk(mu());
    touched_.clear();
    tracking_ = true;
  }
  std::vector<std::pair<void*, size_t>> end_track() {
    std::lock_guard<std::recursive_mutex> lk(mu());
    tracking_ = false;
    std::vector<std::pair<void*, size_t>> v(touched_.begin(), touched_.end());
    touched_.clear();
    return v;
  }
  void pin(const std::vector<std::pair<void*, size_t>>& v) {
    std::lock_guard<std::recursive_mutex> lk(mu());
    for (auto& pb : v) {
      if (pins_[pb.first]++) continue;
      auto fit = free_.find(real(pb.first));  // released during the capture: park it
      if (fit == free_.end()) continue;
      auto& fl = fit->second;
      for (size_t i = 0; i < fl.size(); ++i)
        if (fl[i] == pb.first) {
          fl[i] = fl.back();
          fl.pop_back();
          parked_[pb.first] = real(pb.first);
          break;
        }
      if (fl.empty()) free_.erase(fit);
    }
  }
  void unpin(const std::vector<std::pair<void*, size_t>>& v) {
    std::lock_guard<std::recursive_mutex> lk(mu());
    for (auto& pb : v) {
      auto it = pins_.find(pb.first);
      if (it == pins_.end() || --it->second > 0) continue;
      pins_.erase(it);
      auto pk = parked_.find(pb.first);
      if (pk != parked_.end()) {
        free_[real(pk->first)].push_back(pk->first);
        parked_.erase(pk);
      }
    }
  }
  ~DevicePool() {
    std::lock_guard<std::recursive_mutex> lk(mu());
    for (auto& kv : parked_) free_[real(kv.first)].push_back(kv.first);
    parked_.clear();
    trim();
    stats()[0] -= (double)held_;  // (buffers still handed out are released with their owners)
    auto& r = registry();
    r.erase(std::remove(r.begin(), r.end(), this), r.end());
  }

 private:
  void free_one(void* p) {
    const size_t b = real(p);
    hipFree(p);
    held_ -= b;
    add_held(-(double)b);
    real_.erase(p);
  }
  size_t held_ = 0;
  std::map<size_t, std::vector<void*>> free_;  // allocated size -> cached buffers
  std::unordered_map<void*, size_t> real_;     // every buffer this pool allocated -> its size
  bool tracking_ = false;
  std::unordered_map<void*, size_t> touched_, parked_;
  std::unordered_map<void*, int> pins_;
};

struct Buffer {
  DevicePool* pool;
  u64* p;
  size_t bytes;
  Buffer(DevicePool* pl, size_t b) : pool(pl), p((u64*)pl->alloc(b)), bytes(b) {}
  ~Buffer() { pool->release(p, bytes); }
};

// [ncomp][nlimb][B][N]
struct Poly {
  std::shared_ptr<Buffer> buf;
  int ncomp = 0, nlimb = 0, B = 0, N = 0;
  u64* ptr() const { return buf ? buf->p : nullptr; }
  long long batch_stride() const { return N; }
  long long limb_stride() const { return (long long)B * N; }
  long long comp_stride() const { return (long long)nlimb * B * N; }
};

// an evaluation key made for `level` (common.h key_pos): [digit][2][level+1+K][N]
struct EvKey {
  Poly k;
  int level = 0;
};

struct Ciphertext {
  Poly poly;
  int level = 0;
  long double scale = 1;
  // set when a deferred op that should have written this ciphertext failed:
  // every later use of the handle reports it (deleting it stays possible)
  std::string poison;
  // copy-on-write: handles made by RescaleNew share the rescaled input's
  // buffer (Lattigo returns a copy, evaluator.go:92-99); the first in-place op
  // on either one, while both are alive, copies it first (Context::inplace_ct)
  std::shared_ptr<char> share;
};

struct Plaintext {
  Poly poly;
  int level = 0;
  long double scale = 1;
  bool qp = false;  // limbs: Q 0..level then P (LT diagonals)
};

struct LinTrans {
  int level = 0, N1 = 1;
  float ratio = 1;
  std::vector<int> idx;                 // diagonal indices, as given
  std::map<int, Plaintext> diags;       // keyed by idx & (slots-1)
  std::map<int, Poly> sdiags;           // plan copies for lt_bsgs: limbs below 2^48 stored split24
  std::vector<int> giants, babies;      // sorted giants; babies in first-seen order
  std::map<int, std::vector<int>> index;  // giant -> sorted babies
  // device BSGS plan (built at first evaluation, rebuilt when diagonals change)
  std::vector<int> slots;   // baby of each register slot: nonzero babies, then 0
  std::vector<int> gorder;  // giants in evaluation order: nonzero giants, then 0
  LtPlan* d_plan = nullptr;            // = plan.get()
  std::shared_ptr<void> plan;          // owns d_plan (hipFree); captured graphs hold a reference
  int n_plan = 0;
  bool plan_dirty = true;
  LinTrans() = default;
  LinTrans(const LinTrans&) = delete;
  LinTrans& operator=(const LinTrans&) = delete;
  LinTrans(LinTrans&& o) noexcept { *this = std::move(o); }
  LinTrans& operator=(LinTrans&& o) noexcept {
    level = o.level, N1 = o.N1, ratio = o.ratio;
    idx = std::move(o.idx), diags = std::move(o.diags), giants = std::move(o.giants), babies = std::move(o.babies);
    sdiags = std::move(o.sdiags);
    index = std::move(o.index), slots = std::move(o.slots), gorder = std::move(o.gorder);
    std::swap(d_plan, o.d_plan), std::swap(plan, o.plan), std::swap(n_plan, o.n_plan);
    plan_dirty = o.plan_dirty;
    return *this;
  }
  ~LinTrans() = default;
};

// a handle's context: the scheme's context is 0, pipeline i holds the ids
// [i << 20, (i + 1) << 20)
enum { kCtxShift = 20, kMaxCtx = 64 };
// birth stamps of pooled objects (HandlePool): a pipeline reading another
// context's compiled object orders its stream after the object's producer only
// when the object is younger than what it has already waited for
static std::atomic<unsigned long long> g_birth{1};

template <class T>
class HandlePool {  // lowest-free-id reuse (minheap.go:46-64)
 public:
  // another context's pool, by context index (nullptr: none); and the hook a
  // foreign lookup runs: (owner index, the object's birth stamp, ciphertext?)
  using Resolver = HandlePool<T>* (*)(int owner);
  using Hook = void (*)(int owner, unsigned long long birth);
  static Resolver& resolver() {
    static Resolver r = nullptr;
    return r;
  }
  static Hook& hook() {
    static Hook h = nullptr;
    return h;
  }
  // run on every foreign object get() returns (a capture on the acting
  // context keeps that object's device buffers alive with its graph)
  using Hold = void (*)(const T&);
  static Hold& hold() {
    static Hold h = nullptr;
    return h;
  }
  // run on every object get() returns (a poisoned ciphertext throws)
  using Check = void (*)(const T&);
  static Check& check() {
    static Check c = nullptr;
    return c;
  }
  int add(T&& v) {
    std::lock_guard<std::mutex> lk(mu_);
    int id;
    if (!free_.empty()) {
      id = *free_.begin();
      free_.erase(free_.begin());
    } else {
      id = next_++;
    }
    map_[id] = Entry{std::make_unique<T>(std::move(v)), g_birth.fetch_add(1), false};
    if (born) born->insert(id);
    return id;
  }
  std::set<int>* born = nullptr;  // while set: ids handed out (graph capture)
  // Handles are unique across the contexts of a scheme: an id of another
  // context (a compiled plaintext or transform of the scheme read by a
  // pipeline, a ciphertext handed from one thread to another) resolves to that
  // context's object, after the hook has ordered this thread's stream after
  // the object's producer
  T& get(int id) {
    const int own = id >> kCtxShift;
    if (id >= 0 && own != (base_ >> kCtxShift)) {
      HandlePool* o = resolver() ? resolver()(own) : nullptr;
      if (!o || o == this) throw std::runtime_error("handle not found: " + std::to_string(id));
      unsigned long long birth = 0;
      T& v = o->get_local(id, &birth, true);
      if (check()) check()(v);
      if (hook()) hook()(own, birth);
      if (hold()) hold()(v);
      return v;
    }
    T& v = get_local(id, nullptr);
    if (check()) check()(v);
    return v;
  }
  // a new stamp for an object changed in place (a transform's diagonals)
  void touch(int id) {
    const int own = id >> kCtxShift;
    HandlePool* o = this;
    if (id >= 0 && own != (base_ >> kCtxShift)) o = resolver() ? resolver()(own) : nullptr;
    if (!o) throw std::runtime_error("handle not found: " + std::to_string(id));
    std::lock_guard<std::mutex> lk(o->mu_);
    auto it = o->map_.find(id);
    if (it != o->map_.end()) it->second.birth = g_birth.fetch_add(1);
  }
  bool has(int id) const {
    std::lock_guard<std::mutex> lk(mu_);
    return map_.count(id) != 0;
  }
  // owner of id: this pool, or the pool of the context its id names
  HandlePool* owner_pool(int id) {
    const int own = id >> kCtxShift;
    if (id < 0 || own == (base_ >> kCtxShift)) return this;
    HandlePool* o = resolver() ? resolver()(own) : nullptr;
    return o ? o : this;
  }
  // an object another context has read goes only once the device has drained:
  // that context's kernels may still read its buffer, which the owner's pool
  // would otherwise hand out again in the owner's stream order only
  void del(int id) {
    HandlePool* o = owner_pool(id);
    std::unique_ptr<T> dead;
    {
      std::lock_guard<std::mutex> lk(o->mu_);
      auto it = o->map_.find(id);
      if (it == o->map_.end()) return;
      if (it->second.foreign) (void)hipDeviceSynchronize();
      dead = std::move(it->second.obj);
      o->map_.erase(it);
      o->free_.insert(id);
    }
  }
  void reset() {
    std::lock_guard<std::mutex> lk(mu_);
    map_.clear();
    free_.clear();
    next_ = base_;
  }
  // ids from base on (a pipeline's handles live in a range of their own)
  void set_base(int b) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      base_ = b;
    }
    reset();
  }
  std::vector<int> live() const {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<int> v;
    for (auto& kv : map_) v.push_back(kv.first);
    return v;
  }

 private:
  struct Entry {
    std::unique_ptr<T> obj;
    unsigned long long birth = 0;
    bool foreign = false;  // read by another context
  };
  T& get_local(int id, unsigned long long* birth, bool foreign = false) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = map_.find(id);
    if (it == map_.end()) throw std::runtime_error("handle not found: " + std::to_string(id));
    if (birth) *birth = it->second.birth;
    if (foreign) it->second.foreign = true;
    return *it->second.obj;
  }
  mutable std::mutex mu_;
  std::map<int, Entry> map_;
  std::set<int> free_;
  int base_ = 0, next_ = 0;
};

struct ProfRec {
  int cat;
  hipEvent_t e0, e1;
  double bytes, strict;
};
static const char* kProfNames[] = {"ntt_fwd", "ntt_inv", "elementwise", "basis_ext", "ks_mac", "automorph",
                                   "tensor", "rescale_prep", "lt_bsgs", "lt_giant", "ntt_bext"};
// ntt_bext: forward NTTs whose prologue forms the extended limb (NTT_PRO_BEXT),
// priced (ns + 1) 8 N per limb-transform (+ 8 N for a subtract-and-scale epilogue)
enum { P_NTT_FWD = 0, P_NTT_INV, P_EW, P_BEXT, P_MAC, P_AUT, P_TENSOR, P_RSPREP, P_LTMAC, P_LTGIANT, P_NTT_BEXT, P_NCAT };

// wall-clock intervals of the profiled launches of every context (peer
// pipelines run concurrently), relative to one reference event
// (OrionHipProfileClock): the union per category is the time the GPU spent
// with at least one such launch running (OrionHipProfileUnion)
struct ProfIv {
  int cat;
  float t0, t1;
};
static hipEvent_t g_prof_ref = nullptr;
static std::vector<ProfIv> g_prof_iv;
static std::mutex g_prof_mu;  // g_prof_iv: every context's launches
// ORION_NTT_LOG: one line per NTT call for tools/pmc_summary.py -- one
// line-buffered file for the whole process, so the lines of every context
// (peer pipelines) stay in call order, which is dispatch order
static FILE* ntt_log_file() {
  static FILE* const f = []() -> FILE* {
    const char* p = getenv("ORION_NTT_LOG");
    FILE* h = p && *p ? fopen(p, "a") : nullptr;
    if (h) setvbuf(h, nullptr, _IOLBF, 0);
    return h;
  }();
  return f;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct Context;
static Context* scheme_ctx();  // the scheme's context (index 0), or nullptr

struct Context {
  // index in the scheme's registry (0: the scheme's context, > 0: a pipeline,
  // -1: a bootstrapping context owned by another context); its device; the
  // lock every C-ABI call acting on it holds
  int index = -1, dev = 0;
  std::recursive_mutex mu;
  // per owner context: the birth stamp below which that context's objects are
  // known complete on this context's stream (HandlePool::get's hook)
  unsigned long long synced[kMaxCtx] = {0};
  int logN = 0, N = 0, L = 0, K = 0, dnum = 0, logScale = 0, h = 0;
  // ring (scheme.go:49-52): Standard Z[X]/(X^N + 1), N/2 complex slots, NthRoot
  // 2N; or ConjugateInvariant Z[X + X^-1]/(X^2N + 1) of degree N, N real
  // slots, NthRoot 4N (primes = 1 mod 4N; the NTT folds/unfolds, ntt.hip)
  bool ci = false;
  int slots = 0;
  u64 nthroot = 0;
  std::vector<u64> mods;  // QP
  hipStream_t stream = nullptr;
  bool own_stream = false;
  DevicePool pool;
  DeviceTables host_tb;
  DeviceTables* d_tb = nullptr;
  std::vector<void*> static_bufs;
  double2 *tw_inv = nullptr, *tw_fwd = nullptr;  // special FFT twiddles (encoder.hip)
  std::map<int, u64*> garner;                     // decode CRT tables per level
  Prng prng{0x0123456789abcdefull};               // key generation
  EncSampler enc_sampler;                         // encryption: ChaCha20 key, index, Gaussian table

  Poly sk, pk, rlk;  // rlk: full chain (level L - 1)
  bool have_sk = false, have_pk = false, have_rlk = false;
  // Galois keys, each made for the highest level it has been asked for.  A
  // key covers only the limbs and digits of its level, so a model whose
  // linear transforms run low in the chain (ResNet-20 at N = 2^16: LTs at
  // levels 1-4 under a 48-prime bootstrapping chain) keeps its ~120 keys in
  // a few GB instead of ~150 GB of full-chain keys.
  std::map<u64, EvKey> gks;
  std::map<u64, int> key_hint;  // galEl -> highest level of a linear transform that uses it
  std::map<u64, u32*> autidx;
  std::map<std::pair<int, int>, BasisExtTable*> betab;
  std::map<std::pair<int, int>, std::vector<int>> betab_pos;  // target positions (QP order)
  std::map<int, BasisExtTable*> modup_arr;  // level -> the digits' ModUp tables, contiguous (one device array)

  HandlePool<Plaintext> pts;
  HandlePool<Ciphertext> cts;
  HandlePool<LinTrans> lts;

  // hipGraphs captured from the library stream (OrionHipGraphBegin/End)
  struct GraphRec {
    hipGraph_t g = nullptr;
    hipGraphExec_t x = nullptr;
    std::vector<std::pair<void*, size_t>> pins;
    // every buffer the context's handles, keys and transforms referenced when
    // the capture ended: none of them returns to the pool (and can be handed
    // out again) while the graph may replay, whatever is deleted or replaced
    // meanwhile (DeleteCiphertext, a Galois key made again for a higher level,
    // LoadRotationKey, new LT diagonals or plans, DeleteLinearTransform)
    std::vector<std::shared_ptr<void>> holds;
  };
  std::set<int> capture_born;  // ciphertext ids created inside the open capture
  // buffers of other contexts' objects read inside the open capture (a
  // pipeline's graph reads the scheme's transforms and plaintexts)
  std::vector<std::shared_ptr<void>> capture_holds;
  std::map<int, GraphRec> graphs;
  int next_graph = 0;
  bool capturing = false;
  unsigned prof_saved = 0;

  unsigned prof = 0;  // bit mask of profiled kernel categories
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> ev_free;
  // prof_bytes: the kernel's algorithmic bytes (for the NTT: 16 N per
  // limb-transform + 8 N per epilogue operand or addend it reads, the
  // "fused" model); prof_strict: SURVEY §8d's 16 N per limb-transform alone
  double prof_launch[P_NCAT] = {0}, prof_ms[P_NCAT] = {0}, prof_bytes[P_NCAT] = {0}, prof_strict[P_NCAT] = {0};

  ~Context() {
    hipDeviceSynchronize();
    btps.clear();  // circuits first: their buffers belong to the bootstrapping contexts' pools
    btp_ctx.clear();
    if (capturing) {
      hipGraph_t gr = nullptr;
      hipStreamEndCapture(stream, &gr);
      if (gr) hipGraphDestroy(gr);
    }
    for (auto& kv : graphs) {
      hipGraphExecDestroy(kv.second.x);
      hipGraphDestroy(kv.second.g);
    }
    graphs.clear();
    gks.clear();
    sk = pk = rlk = Poly();
    pts.reset();
    cts.reset();
    lts.reset();
    for (auto& kv : autidx) hipFree(kv.second);
    for (auto& kv : betab) hipFree(kv.second);
    for (auto& kv : modup_arr) hipFree(kv.second);
    for (auto& kv : garner) hipFree(kv.second);
    for (void* p : static_bufs) hipFree(p);
    if (d_tb) hipFree(d_tb);
    for (auto& r : prof_recs) {
      hipEventDestroy(r.e0);
      hipEventDestroy(r.e1);
    }
    for (auto e : ev_free) hipEventDestroy(e);
    for (auto e : cs_ev)
      if (e) hipEventDestroy(e);
    for (auto s : cs_stream)
      if (s) hipStreamDestroy(s);
    if (own_stream && stream) hipStreamDestroy(stream);
  }

  // -- profiling -----------------------------------------------------------
  hipEvent_t ev() {
    if (!ev_free.empty()) {
      hipEvent_t e = ev_free.back();
      ev_free.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    return e;
  }
  struct Scope {
    Context* c;
    int cat;
    double bytes, strict;
    hipEvent_t e0 = nullptr;
    Scope(Context* ctx, int k, double b, double st = -1) : c(ctx), cat(k), bytes(b), strict(st < 0 ? b : st) {
      if (c->prof & (1u << cat)) {
        e0 = c->ev();
        hipEventRecord(e0, c->stream);
      }
    }
    ~Scope() {
      if (e0) {
        hipEvent_t e1 = c->ev();
        hipEventRecord(e1, c->stream);
        c->prof_recs.push_back(ProfRec{cat, e0, e1, bytes, strict});
        if (c->prof_recs.size() > 20000) c->prof_flush();
      }
    }
  };
  void prof_flush() {
    if (prof_recs.empty()) return;
    hipStreamSynchronize(stream);
    for (auto& r : prof_recs) {
      float ms = 0;
      hipEventElapsedTime(&ms, r.e0, r.e1);
      if (g_prof_ref) {
        float a0 = 0, a1 = 0;
        hipEventElapsedTime(&a0, g_prof_ref, r.e0);
        hipEventElapsedTime(&a1, g_prof_ref, r.e1);
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof_iv.push_back(ProfIv{r.cat, a0, a1});
      }
      prof_launch[r.cat] += 1;
      prof_ms[r.cat] += ms;
      prof_bytes[r.cat] += r.bytes;
      prof_strict[r.cat] += r.strict;
      ev_free.push_back(r.e0);
      ev_free.push_back(r.e1);
    }
    prof_recs.clear();
  }

  // -- graph capture ---------------------------------------------------------------
  // Every op issued between graph_begin and graph_end is recorded (not run)
  // into one hipGraph; a replay re-runs all its kernels on the library stream
  // with one launch.  The captured ops must not synchronise (keys, tables and
  // LT plans are made by a warm-up pass first); profiling is off meanwhile.
  void graph_begin() {
    if (capturing) throw std::runtime_error("a graph capture is already open");
    HIPCHK(hipStreamSynchronize(stream));
    prof_flush();
    prof_saved = prof;
    prof = 0;
    pool.begin_track();
    capture_born.clear();
    capture_holds.clear();
    cts.born = &capture_born;
    HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
    capturing = true;
  }
  int graph_end() {
    if (!capturing) throw std::runtime_error("no graph capture is open");
    capturing = false;
    cts.born = nullptr;
    prof = prof_saved;
    hipGraph_t gr = nullptr;
    const hipError_t e = hipStreamEndCapture(stream, &gr);
    auto touched = pool.end_track();
    if (e != hipSuccess || !gr) {
      if (gr) hipGraphDestroy(gr);
      pool.unpark_unpinned(touched);
      // an invalidated capture leaves its stream unusable: end whatever is
      // still open and, for the library's own stream, start a fresh one
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
        hipGraph_t g2 = nullptr;
        hipStreamEndCapture(stream, &g2);
        if (g2) hipGraphDestroy(g2);
      }
      (void)hipGetLastError();
      if (own_stream) {
        hipStreamDestroy(stream);
        HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
      }
      throw std::runtime_error(std::string("graph capture failed (an op synchronised or left the stream?): ") +
                               hipGetErrorString(e));
    }
    GraphRec r;
    r.g = gr;
    const hipError_t ei = hipGraphInstantiate(&r.x, gr, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      hipGraphDestroy(gr);
      pool.unpark_unpinned(touched);
      throw std::runtime_error(std::string("graph instantiation failed: ") + hipGetErrorString(ei));
    }
    pool.pin(touched);
    r.pins = std::move(touched);
    r.holds = graph_holds();
    r.holds.insert(r.holds.end(), capture_holds.begin(), capture_holds.end());
    capture_holds.clear();
    const int id = next_graph++;
    graphs[id] = std::move(r);
    return id;
  }
  void graph_launch(int id) {
    auto it = graphs.find(id);
    if (it == graphs.end()) throw std::runtime_error("graph not found: " + std::to_string(id));
    if (capturing) throw std::runtime_error("graph launch while capturing");
    HIPCHK(hipGraphLaunch(it->second.x, stream));
  }
  void graph_destroy(int id) {
    auto it = graphs.find(id);
    if (it == graphs.end()) return;
    HIPCHK(hipStreamSynchronize(stream));
    hipGraphExecDestroy(it->second.x);
    hipGraphDestroy(it->second.g);
    pool.unpin(it->second.pins);
    graphs.erase(it);
  }

  std::vector<std::shared_ptr<void>> graph_holds() {
    std::vector<std::shared_ptr<void>> h;
    auto add = [&h](const Poly& p) {
      if (p.buf) h.push_back(p.buf);
    };
    add(sk), add(pk), add(rlk);
    for (auto& kv : gks) add(kv.second.k);
    for (int id : cts.live()) add(cts.get(id).poly);
    for (int id : pts.live()) add(pts.get(id).poly);
    for (int id : lts.live()) {
      LinTrans& t = lts.get(id);
      for (auto& kv : t.diags) add(kv.second.poly);
      for (auto& kv : t.sdiags) add(kv.second);
      if (t.plan) h.push_back(t.plan);
    }
    return h;
  }
  // in-place ops inside a capture only on ciphertexts made inside it: on an
  // older handle a replay would apply the op again to its own output, and the
  // handle's level and scale would advance once (at capture) while its data
  // changes at every launch
  // a ciphertext an op is about to modify in place; cow = false: the caller
  // replaces the whole buffer (no copy of a shared one is needed)
  Ciphertext& inplace_ct(int id, bool cow = true) {
    // a buffer replaced here goes back to its owner's pool, which hands out
    // buffers in its own stream's order only: another context's ciphertext is
    // read, never changed
    if (index >= 0 && id >= 0 && (id >> kCtxShift) != index)
      throw std::runtime_error("in-place op on ciphertext " + std::to_string(id) + " of pipeline " +
                               std::to_string(id >> kCtxShift) + " from pipeline " + std::to_string(index) +
                               ": a ciphertext is changed only by the context (thread) that made it");
    Ciphertext& a = cts.get(id);
    if (capturing && !capture_born.count(id))
      throw std::runtime_error("in-place op on ciphertext " + std::to_string(id) +
                               ", which predates the graph capture (a replay would reapply it): clone it inside the "
                               "capture first");
    if (cow && a.share) {
      if (a.share.use_count() > 1) a.poly = clone(a).poly;  // the other handle keeps the old buffer
      a.share.reset();
    }
    return a;
  }
  // RescaleNew's result: a second handle on a's (just rescaled) buffer, when
  // nothing else (a captured graph) holds that buffer
  Ciphertext alias(Ciphertext& a) {
    if (!defer_on || !a.poly.buf || a.poly.buf.use_count() != 1) return clone(a);
    if (!a.share) a.share = std::make_shared<char>(0);
    Ciphertext y;
    y.poly = a.poly;
    y.level = a.level;
    y.scale = a.scale;
    y.share = a.share;
    return y;
  }

  // -- deferred rotate-and-add, behind the unchanged C-ABI -------------------
  // The frontend's `out += out.roll(k)` (linear.py:72-73 -> tensors.py:244-258,
  // :139-167) issues RotateNew(x, k) -> r, AddCiphertext(x, r) and, when the
  // temporary CipherTensor dies, DeleteCiphertext(r).  RotateNew only records
  // the rotation (r gets its metadata, no buffer); the AddCiphertext that adds
  // r into its own source records the sum; when r is then deleted unread, the
  // pair runs as one key switch whose ModDown store adds into x
  // (rotate_add_inplace), and r's contents are never formed.  Any other C-ABI
  // call first runs what is pending as the op-by-op path would (defer_flush
  // at the API layer).  ORION_DEFER=0 turns this and RescaleNew's aliasing off.
  struct Deferred {
    int kind = 0;  // 1: r = Rotate(x, k) pending; 2: and x += r pending
    int x = -1, r = -1, k = 0;
  };
  Deferred dfr;
  bool defer_on = getenv("ORION_DEFER") ? atoi(getenv("ORION_DEFER")) != 0 : true;

  // lazily built tables, keys and host transfers synchronise, which would
  // invalidate an open capture (and leave HIP's stream state unusable): refuse
  // them first
  void no_capture(const char* what) const {
    if (capturing)
      throw std::runtime_error(std::string(what) +
                               " needs a host synchronisation, not allowed while capturing a graph (run the op "
                               "stream once before capturing it)");
  }
  // tables and plans made on first use go to the device in the library
  // stream's order: a blocking hipMemcpy runs on the legacy NULL stream, which
  // the non-blocking library stream does not wait for (a device-to-device
  // hipMemcpy can even return before the copy lands), so a kernel queued next
  // could read a table the copy has not finished, and a rewritten plan could
  // change under a kernel still queued on the stream
  void h2d(void* d, const void* h, size_t n) {
    HIPCHK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }

  // -- allocation --------------------------------------------------------------
  Poly alloc(int ncomp, int nlimb, int B) {
    Poly p;
    p.ncomp = ncomp;
    p.nlimb = nlimb;
    p.B = B;
    p.N = N;
    p.buf = std::make_shared<Buffer>(&pool, (size_t)ncomp * nlimb * B * N * sizeof(u64) + 16);
    return p;
  }

  int qp_mod(int level, int pos) const { return pos <= level ? pos : L + (pos - level - 1); }

  // LimbSet over components [c0, c0+nc) and limb positions/moduli
  LimbSet ls(const Poly& P, int c0, int nc, const std::vector<int>& pos, const std::vector<int>& md,
             int nbatch = -1) const {
    LimbSet s;
    memset(&s, 0, sizeof(s));
    s.p = P.ptr() + c0 * P.comp_stride();
    s.comp_stride = P.comp_stride();
    s.limb_stride = P.limb_stride();
    s.batch_stride = P.batch_stride();
    s.ncomp = nc;
    s.nlimb = (int)pos.size();
    s.nbatch = nbatch < 0 ? P.B : nbatch;
    if (P.B == 1 && s.nbatch > 1) s.batch_stride = 0;  // broadcast
    if (pos.size() > ORION_MAXLIMB) throw std::runtime_error("too many limbs in one launch");
    for (size_t i = 0; i < pos.size(); ++i) {
      s.pos[i] = (unsigned char)pos[i];
      s.mod[i] = (unsigned char)md[i];
    }
    return s;
  }
  static std::vector<int> iota(int a, int b) {
    std::vector<int> v;
    for (int i = a; i < b; ++i) v.push_back(i);
    return v;
  }
  LimbSet lsq(const Poly& P, int c0, int nc, int level, int nbatch = -1) const {
    auto v = iota(0, level + 1);
    return ls(P, c0, nc, v, v, nbatch);
  }
  // QP limbs of a poly laid out [Q 0..lvl_alloc][P], used at `level` <= lvl_alloc
  LimbSet lsqp(const Poly& P, int c0, int nc, int level, int lvl_alloc, int nbatch = -1) const {
    std::vector<int> pos, md;
    for (int j = 0; j <= level; ++j) pos.push_back(j), md.push_back(j);
    for (int k = 0; k < K; ++k) pos.push_back(lvl_alloc + 1 + k), md.push_back(L + k);
    return ls(P, c0, nc, pos, md, nbatch);
  }
  LimbSet lsp(const Poly& P, int c0, int nc, int lvl_alloc) const {
    std::vector<int> pos, md;
    for (int k = 0; k < K; ++k) pos.push_back(lvl_alloc + 1 + k), md.push_back(L + k);
    return ls(P, c0, nc, pos, md);
  }

  // -- kernel wrappers ------------------------------------------------------------
  // NTT / INTT with a fused prologue (load, basis extension, rescale prep) and
  // epilogue (store, subtract-and-scale); bytes: 16 N per limb-transform
  static NttIO nio(const LimbSet& dst, const LimbSet& src) {
    NttIO io;
    memset(&io, 0, sizeof(io));
    io.dst = dst;
    io.src = src;
    return io;
  }
#ifndef ORION_NTT_DEFAULT_ORDER
#define ORION_NTT_DEFAULT_ORDER 2
#endif
  int ntt_order = getenv("ORION_NTT_ORDER") ? atoi(getenv("ORION_NTT_ORDER")) : ORION_NTT_DEFAULT_ORDER;
#ifndef ORION_NTT_DEFAULT_IMPL
#define ORION_NTT_DEFAULT_IMPL 1
#endif
  // 1: one limb per workgroup (ntt.hip); 2: two-pass N = 2^15 kernels (ntt2.hip)
  int ntt_impl = getenv("ORION_NTT_IMPL") ? atoi(getenv("ORION_NTT_IMPL")) : ORION_NTT_DEFAULT_IMPL;
  // two-pass kernels: limb-transforms per chunk (0 = one launch pair for all)
  int ntt2_chunk = getenv("ORION_NTT2_CHUNK") ? atoi(getenv("ORION_NTT2_CHUNK")) : 0;
  // N = 2^15 launches with fewer limb-transforms than this use the two-pass
  // kernels: one limb per CU leaves most of the 256 CUs idle there (8 jobs:
  // 15 vs 37 us; 64 jobs: 32 vs 40 us, float64 path).  Batched launches
  // (>= 128 jobs at 64 images) keep the one-pass kernel.
  int ntt2_below = getenv("ORION_NTT2_BELOW") ? atoi(getenv("ORION_NTT2_BELOW")) : 128;
  // two-pass launches of at most this many limb-transforms use the
  // latency-oriented kernels of ntt2s.hip (one butterfly per thread per
  // stage, the tile in LDS) instead of ntt2.hip's 16-point threads
  int ntt2s_below = getenv("ORION_NTT2S_BELOW") ? atoi(getenv("ORION_NTT2S_BELOW")) : 128;
  // decompositions with fewer limb-transforms per digit than this run every
  // digit's ModUp + NTT as one launch pair (0 = always per digit)
  int modup_merge = getenv("ORION_MODUP_MERGE") ? atoi(getenv("ORION_MODUP_MERGE")) : 256;
  // 1: ModUp and ModDown form the extended limbs in the forward NTT's prologue
  // (NTT_PRO_BEXT) instead of a basis_ext / modup_all launch whose output the
  // NTT reads back (sources of at most 2 limbs, Standard ring), when the NTT
  // runs on the two-pass kernels (fuse_bext); 2: on the one-pass kernel too
  // (timing switch); 0: never
  int bext_fuse = getenv("ORION_BEXT_FUSE") ? atoi(getenv("ORION_BEXT_FUSE")) : 1;
  // N = 2^15 inverse launches up to ntt2_tail_max limb-transforms whose last
  // round of one-limb workgroups would be partial (jobs / (rounds * CUs) below
  // ntt2_tail_eff) also take the two-pass kernels: a one-pass round costs one
  // limb's latency on every CU whether or not the CU has a job, while the
  // two-pass kernels scale with the job count (tools/ntt_bench.py, mixed
  // moduli, inverse: 192 jobs 61 vs 76 us, 384 jobs 98 vs 127 us).  Forward
  // launches keep the one-pass kernel: their fused epilogues cost the
  // two-pass kernels a scratch round trip, and the LoLA bench measured them
  // slower (profiles/r01z_ntt2_tailfwd_ab.txt)
  double ntt2_tail_eff = getenv("ORION_NTT2_TAIL_EFF") ? atof(getenv("ORION_NTT2_TAIL_EFF")) : 0.9;
  int ntt2_tail_max = getenv("ORION_NTT2_TAIL_MAX") ? atoi(getenv("ORION_NTT2_TAIL_MAX")) : 1024;
  // 1: plain forward launches (load prologue, store epilogue) follow the same
  // rule; 2: every forward launch that needs no scratch (not an in-place tail)
  int ntt2_tail_fwd = getenv("ORION_NTT2_TAIL_FWD") ? atoi(getenv("ORION_NTT2_TAIL_FWD")) : 1;
  int n_cu = 0;
  int cus() {
    if (n_cu == 0) {
      int dev = 0;
      HIPCHK(hipGetDevice(&dev));
      HIPCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    return n_cu;
  }
  bool ntt2_tail(int jobs) {
    if (jobs > ntt2_tail_max || ntt2_tail_eff <= 0) return false;
    cus();
    const int rounds = (jobs + n_cu - 1) / n_cu;
    return (double)jobs / ((double)rounds * n_cu) < ntt2_tail_eff;
  }
  // timing switches: s_sleep(127) iterations (~3.4 us each) before the first
  // job of every other CU in persistent launches of >= ntt_stagger_min rounds
  int ntt_stagger = getenv("ORION_NTT_STAGGER") ? atoi(getenv("ORION_NTT_STAGGER")) : 0;
  int ntt_stagger_min = getenv("ORION_NTT_STAGGER_MIN") ? atoi(getenv("ORION_NTT_STAGGER_MIN")) : 2;
  // co-split (timing switch): a one-pass launch of >= ntt_cosplit_min jobs
  // gives the fraction ntt_cosplit of its jobs (its tail: the float64 limbs
  // under job order 2) to the two-pass kernels, run concurrently on a
  // disjoint set of CUs: the one-pass kernel is bound by one job per CU with
  // serialised phases (~45% of HBM streaming), the two-pass kernels by HBM
  // (86-89%), so the two can share the chip.  ntt_cosplit_q quarters of every
  // XCD's CUs take the one-pass part (CU-masked streams, joined to the
  // context's stream by events)
  double ntt_cosplit = getenv("ORION_NTT_COSPLIT") ? atof(getenv("ORION_NTT_COSPLIT")) : 0.0;
  int ntt_cosplit_min = getenv("ORION_NTT_COSPLIT_MIN") ? atoi(getenv("ORION_NTT_COSPLIT_MIN")) : 512;
  int ntt_cosplit_q = getenv("ORION_NTT_COSPLIT_Q") ? atoi(getenv("ORION_NTT_COSPLIT_Q")) : 2;
  hipStream_t cs_stream[2] = {nullptr, nullptr};
  hipEvent_t cs_ev[3] = {nullptr, nullptr, nullptr};
  int cs_cus = 0;  // CUs of the one-pass side
  void cosplit_init() {
    if (cs_stream[0]) return;
    const int n = cus(), words = (n + 31) / 32;
    // bit i in the one-pass set when (i / 8) % 4 < q: a quarter-granular share
    // of every XCD whether the mask's CUs are numbered XCD-major or interleaved
    std::vector<uint32_t> ma(words, 0), mb(words, 0);
    cs_cus = 0;
    for (int i = 0; i < n; ++i) {
      const bool a = (i / 8) % 4 < ntt_cosplit_q;
      (a ? ma : mb)[i / 32] |= 1u << (i % 32);
      cs_cus += a;
    }
    HIPCHK(hipExtStreamCreateWithCUMask(&cs_stream[0], words, ma.data()));
    HIPCHK(hipExtStreamCreateWithCUMask(&cs_stream[1], words, mb.data()));
    for (auto& e : cs_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // ORION_NTT_LOG=path: one line per NTT call ("<dispatches> <jobs> <epi> <inv>
  // <pro> <intjobs> <family>": dispatches = kernel launches of the call (1 or
  // 2); epi = the epilogue (NTT_EPI_*); pro = the prologue; intjobs =
  // limb-transforms on integer-path (>= 2^46) moduli; family 1 = ntt.hip, 2 =
  // ntt2.hip, 3 = ntt2s.hip, 4 = an ntt2s.hip INTT's rows pass alone), so
  // tools/pmc_summary.py can price each dispatch of a rocprofv3 pass with its
  // limb-transform count (persistent launches have fewer workgroups than
  // jobs) and break the NTT time down by launch class
  void log_ntt(int family, const NttIO& io, bool inv) {
    FILE* const ntt_log = ntt_log_file();
    if (!ntt_log) return;
    int nint = 0;
    for (int l = 0; l < io.dst.nlimb; ++l) nint += host_tb.mc[io.dst.mod[l]].f64 ? 0 : 1;
    const int dispatches = family == 2 || family == 3 ? 2 : 1;
    fprintf(ntt_log, "%d %d %d %d %d %d %d\n", dispatches, io.jobs, io.epi, inv ? 1 : 0,
            io.pro, io.jobs / std::max(1, io.dst.nlimb) * nint, family);
  }
  // whether an NTT launch of `jobs` limb-transforms runs on the two-pass
  // kernels (ntt2.hip): N = 2^16 always; N = 2^15 for small launches and for
  // partial last rounds of inverse and plain forward launches (see above)
  bool two_pass(int jobs, bool inv, int pro, int epi, bool inplace_sub) {
    if (logN == 16) return true;
    if (logN != 15 || ci) return false;
    if (md_force) return true;
    if (ntt_impl == 2 || jobs < ntt2_below) return true;
    const bool plain = (pro == NTT_PRO_LOAD || pro == NTT_PRO_BEXT) && epi == NTT_EPI_STORE;
    return (inv || (ntt2_tail_fwd == 1 && plain) || (ntt2_tail_fwd == 2 && !inplace_sub) ||
            (ntt2_tail_aut && epi_aut(epi) && pro == NTT_PRO_LOAD)) &&
           ntt2_tail(jobs);
  }
  // 1: the partial-round rule above also moves the rotations' scatter-store
  // ModDown NTTs (NTT_EPI_SUBSCALE_AUT[_ACC]) onto the two-pass kernels
  int ntt2_tail_aut = getenv("ORION_NTT2_TAIL_AUT") ? atoi(getenv("ORION_NTT2_TAIL_AUT")) : 0;
  // the fused basis extension (NTT_PRO_BEXT) pays on the two-pass kernels
  // only: in the one-pass kernel, one CU per limb, every target re-forms the
  // shared y_i and float quotient and loads ns source limbs in its memory
  // phase, and the LoLA step took 36.8 instead of 30.6 ms
  // (profiles/r04c_bext_fuse_ab.txt); on the two-pass kernels batch 1 went
  // from 3.0 to 2.84 ms per image
  // and at B = 64 LoLA its partial-round two-pass launches were neutral to
  // -0.5% (2089 / 2091 vs 2105 / 2097 img/s, profiles/r04d_bext_fuse_ab.txt),
  // so it is kept to small launches (bext_fuse_below limb-transforms)
  bool fuse_bext(int jobs, int ns, int epi) {
    if (!bext_fuse || ns > 2 || ci) return false;
    return bext_fuse == 2 || ((md_force || jobs <= bext_fuse_below) && two_pass(jobs, false, NTT_PRO_BEXT, epi, false));
  }
  // timing switch ORION_MODDOWN_LAT=1 (2: rotations only): every ModDown takes the fused latency
  // path whatever its size (the gadget product's rows pass of the P limbs'
  // INTT, their columns pass + the extension + the Q limbs' forward columns in
  // ntt2s_ifwd_cols_p, the Q rows pass with the subtract-and-scale), instead of
  // the one-pass INTT, basis_ext and one-pass NTT of large batches.  md_force
  // holds while a ModDown (or its fusability test) decides its launches
  int moddown_lat = getenv("ORION_MODDOWN_LAT") ? atoi(getenv("ORION_MODDOWN_LAT")) : 0;
  bool md_force = false;
  struct MdForce {
    Context* c;
    bool old;
    // (2: only the rotations' ModDowns, whose one-pass scatter-store NTT is the slowest class)
    MdForce(Context* c_, bool aut) : c(c_), old(c_->md_force) {
      c->md_force = !c->ci && (c->moddown_lat == 1 || (c->moddown_lat == 2 && aut));
    }
    ~MdForce() { c->md_force = old; }
  };
  int bext_fuse_below = getenv("ORION_BEXT_FUSE_BELOW") ? atoi(getenv("ORION_BEXT_FUSE_BELOW")) : 64;
  // src_per_job: NTT_PRO_BEXT launches, the mean source limbs read per
  // limb-transform (their algorithmic bytes are (src_per_job + 1) 8 N, + 8 N
  // for a subtract-and-scale epilogue, in the ntt_bext category)
  void prep_io(NttIO& io) {
    io.order = ntt_order;
    io.ci = ci ? 1 : 0;
    io.jobs = io.dst.ncomp * io.dst.nlimb * io.dst.nbatch;
    if (io.order == 2) {  // integer-path (>= 2^46) limbs are ~1.4x slower per transform: dispatch them first
      int k = 0;
      for (int pass = 0; pass < 2; ++pass)
        for (int l = 0; l < io.dst.nlimb; ++l)
          if ((host_tb.mc[io.dst.mod[l]].f64 != 0) == (pass == 1)) io.lord[k++] = (unsigned char)l;
    }
  }
  // 1: an INTT whose output feeds only the prologue of the forward NTT that
  // follows (ModUp and ModDown sources, the rescale's last limb) runs its rows
  // pass alone when both launches take the latency kernels (ntt2s.hip); the
  // forward launch finishes the INTT's columns pass on its own column tile
  // (ntt2s_ifwd_cols), so the INTT output never goes to HBM and its second
  // launch disappears
  int ntt_ifuse = getenv("ORION_NTT_IFUSE") ? atoi(getenv("ORION_NTT_IFUSE")) : 1;
  // 1: a rotation's NTT-domain automorphism is applied in the ModDown's final
  // NTT store (NTT_EPI_SUBSCALE_AUT) where the kernel supports it
  int ntt_aut_fuse = getenv("ORION_NTT_AUT_FUSE") ? atoi(getenv("ORION_NTT_AUT_FUSE")) : 1;
  // 1: a one-pass launch whose last round of one-limb workgroups is partial
  // (at most ntt_tailsplit_max jobs) runs its whole rounds on the one-pass
  // kernel and the partial round on the two-pass kernels
  int ntt_tailsplit = getenv("ORION_NTT_TAILSPLIT") ? atoi(getenv("ORION_NTT_TAILSPLIT")) : 0;
  int ntt_tailsplit_max = getenv("ORION_NTT_TAILSPLIT_MAX") ? atoi(getenv("ORION_NTT_TAILSPLIT_MAX")) : 160;
  // ... as long as the sources' columns pass is not redone too often: every
  // target workgroup redoes it for its own sources, (targets x sources per
  // target) / source limbs times the INTT's own columns work (ResNet's
  // N = 2^16 ModDowns onto 20-30 Q limbs measured slower fused)
  double ntt_ifuse_maxr = getenv("ORION_NTT_IFUSE_MAXR") ? atof(getenv("ORION_NTT_IFUSE_MAXR")) : 8.0;
  // 2 or 4: the fused forward runs a workgroup of that many 256-thread groups
  // per segment of targets sharing their sources, which finishes the sources'
  // INTT columns once for the segment (ntt2s_ifwd_cols_p); 1: one target per
  // workgroup, the sources' columns redone for each (ntt2s_ifwd_cols)
  int ntt_ifuse_p = getenv("ORION_NTT_IFUSE_P") ? atoi(getenv("ORION_NTT_IFUSE_P")) : 2;
  bool on_ntt2s(int jobs, bool inv, int pro, int epi, bool inplace_sub) {
    return (logN == 15 || logN == 16) && !ci && (md_force || jobs <= ntt2s_below) &&
           two_pass(jobs, inv, pro, epi, inplace_sub);
  }
  // the INTT iio (load prologue, store epilogue) and then the forward fio whose
  // BEXT / RESCALE prologue reads the INTT's output (fio.src = iio.dst); ns_max:
  // the most source limbs one target reads
  // whether intt_then_fwd(iio, fio, ns_max) takes the fused path (the INTT's
  // rows pass alone, its columns pass inside the forward's latency kernels)
  bool ifuse_ok(const NttIO& iio, const NttIO& fio, int ns_max) {
    const int ij = iio.dst.ncomp * iio.dst.nlimb * iio.dst.nbatch;
    const int fj = fio.dst.ncomp * fio.dst.nlimb * fio.dst.nbatch;
    bool same = iio.dst.p == fio.src.p && iio.dst.nlimb == fio.src.nlimb && iio.dst.ncomp == fio.src.ncomp &&
                iio.dst.nbatch == fio.src.nbatch && iio.dst.comp_stride == fio.src.comp_stride &&
                iio.dst.limb_stride == fio.src.limb_stride && iio.dst.batch_stride == fio.src.batch_stride;
    for (int l = 0; same && l < iio.dst.nlimb; ++l)
      same = iio.dst.pos[l] == fio.src.pos[l] && iio.dst.mod[l] == fio.src.mod[l];
    const bool inplace_sub = fio.epi != NTT_EPI_STORE && fio.ex.p == fio.dst.p;
    const double redo = (double)fio.dst.nlimb * ns_max / std::max(1, iio.dst.nlimb);
    return ntt_ifuse && redo <= ntt_ifuse_maxr && same && iio.pro == NTT_PRO_LOAD && iio.epi == NTT_EPI_STORE &&
           (fio.pro == NTT_PRO_BEXT || fio.pro == NTT_PRO_RESCALE) &&
           on_ntt2s(ij, true, NTT_PRO_LOAD, NTT_EPI_STORE, false) && on_ntt2s(fj, false, fio.pro, fio.epi, inplace_sub);
  }
  // rows_done: the caller's kernel already stored the INTT's rows-pass
  // intermediate in iio.dst (ks_mac_rows_kernel); only the fused path is valid then
  void intt_then_fwd(NttIO iio, NttIO fio, int ns_max, double src_per_job = 0, bool rows_done = false) {
    if (!ifuse_ok(iio, fio, ns_max)) {
      if (rows_done) throw std::runtime_error("NTT: rows pass done, but the fused forward is not available");
      ntt_io(iio, true);
      ntt_io(fio, false, src_per_job);
      return;
    }
    const int ij = iio.dst.ncomp * iio.dst.nlimb * iio.dst.nbatch;
    prep_io(iio);
    iio.mid = iio.dst;  // the rows pass leaves its intermediate in the INTT's own output rows
    if (!rows_done) {
      Scope sc(this, P_NTT_INV, 16.0 * N * ij);
      if (orion_launch_ntt2s(logN, iio, d_tb, true, stream, true)) throw std::runtime_error("NTT launch failed");
      log_ntt(4, iio, true);
    }
    fio.ifuse = 1;
    fio.imid = iio.dst;
    if (NTT2S_R4 && (ntt_ifuse_p == 2 || ntt_ifuse_p == 4)) {
      // segments: runs of target limbs on the same basis-extension table (the
      // same source limbs; the rescale prep has one source), at most G each
      int k = 0;
      for (int l = 0; l < fio.dst.nlimb;) {
        int e = l + 1;
        while (e < fio.dst.nlimb && e - l < ntt_ifuse_p &&
               (fio.pro != NTT_PRO_BEXT || fio.bx_tab[e] == fio.bx_tab[l]))
          ++e;
        fio.tg_l0[k] = (unsigned char)l;
        fio.tg_n[k] = (unsigned char)(e - l);
        ++k;
        l = e;
      }
      fio.ntg = k;
      fio.tgroup = ntt_ifuse_p;
    }
    ntt_io(fio, false, src_per_job);
  }
  void ntt_io(NttIO io, bool inv, double src_per_job = 0) {
    prep_io(io);
    const bool bx = io.pro == NTT_PRO_BEXT;
    // fused model: + 8 N for the subtract-and-scale operand, + 8 N for the word
    // a rotate-and-add store adds to; an automorphism's scatter index is a
    // table shared by every limb and image of the Galois element, amortised
    // like the twiddles and not counted.  strict: 16 N per
    // limb-transform, whatever the prologue and epilogue read
    const double per = (bx ? (src_per_job + 1) * 8.0 * N : 16.0 * N) + (io.epi != NTT_EPI_STORE ? 8.0 * N : 0.0) +
                       (io.epi == NTT_EPI_SUBSCALE_AUT_ACC ? 8.0 * N : 0.0);
    const double strict = 16.0 * N;
    const int cat = bx ? P_NTT_BEXT : inv ? P_NTT_INV : P_NTT_FWD;
    if (two_pass(io.jobs, inv, io.pro, io.epi, io.epi != NTT_EPI_STORE && io.ex.p == io.dst.p)) {
      Poly scratch;
      // large launches in chunks of jobs through one reused compact scratch
      // (the intermediate can stay in the Infinity Cache); the latency
      // kernels' small launches are never chunked
      if (ntt2_chunk > 0 && io.jobs > std::max(ntt2_chunk, ntt2s_below) && !io.ifuse) {
        const int chunk = std::min(ntt2_chunk, io.jobs);
        scratch = alloc(1, 1, chunk);
        io.mid = ls(scratch, 0, 1, {0}, {0});
        io.mid_compact = 1;
        Scope sc(this, cat, per * io.jobs, strict * io.jobs);
        for (int j0 = 0; j0 < io.jobs; j0 += chunk) {
          io.job0 = j0;
          io.njob = std::min(chunk, io.jobs - j0);
          if (orion_launch_ntt2(logN, io, d_tb, inv, stream)) throw std::runtime_error("NTT launch failed");
          NttIO lio = io;
          lio.jobs = io.njob;
          log_ntt(2, lio, inv);
        }
        return;
      }
      io.mid = io.dst;
      // in-place tail: keep ex intact for pass 2; automorphism epilogue: a rows
      // workgroup stores into other rows of dst (and, accumulating, reads
      // their old words), so the intermediate cannot live there
      if ((io.epi != NTT_EPI_STORE && io.ex.p == io.dst.p) || epi_aut(io.epi)) {
        scratch = alloc(io.dst.ncomp, io.dst.nlimb, io.dst.nbatch);
        io.mid = ls(scratch, 0, io.dst.ncomp, iota(0, io.dst.nlimb), std::vector<int>(io.dst.mod, io.dst.mod + io.dst.nlimb));
      }
      Scope sc(this, cat, per * io.jobs, strict * io.jobs);
      const bool small = md_force || io.jobs <= ntt2s_below;
      if (io.ifuse && !small) throw std::runtime_error("NTT: a fused INTT columns pass needs the latency kernels");
      if (small ? orion_launch_ntt2s(logN, io, d_tb, inv, stream) : orion_launch_ntt2(logN, io, d_tb, inv, stream))
        throw std::runtime_error("NTT launch failed");
      log_ntt(small ? 3 : 2, io, inv);
      return;
    }
    if (io.ifuse) throw std::runtime_error("NTT: a fused INTT columns pass needs the latency kernels");
    cus();
    if (ntt_cosplit > 0 && logN == 15 && !ci && io.jobs >= ntt_cosplit_min && !capturing) {
      // jobs [0, j1) on the one-pass kernel (one persistent workgroup per CU
      // of its share), jobs [j1, jobs) on the two-pass kernels through a
      // compact scratch, concurrently on the two CU-masked streams
      cosplit_init();
      const int j2 = std::min(io.jobs - 1, std::max(1, (int)lround(io.jobs * ntt_cosplit))), j1 = io.jobs - j2;
      Scope sc(this, cat, per * io.jobs, strict * io.jobs);
      Poly scratch = alloc(1, 1, j2);
      NttIO a = io;
      a.njob = j1;
      a.grid = cs_cus;
      NttIO b = io;
      b.mid = ls(scratch, 0, 1, {0}, {0});
      b.mid_compact = 1;
      b.job0 = j1;
      b.njob = j2;
      HIPCHK(hipEventRecord(cs_ev[0], stream));
      HIPCHK(hipStreamWaitEvent(cs_stream[0], cs_ev[0], 0));
      HIPCHK(hipStreamWaitEvent(cs_stream[1], cs_ev[0], 0));
      if (orion_launch_ntt_io(logN, a, d_tb, inv, cs_stream[0])) throw std::runtime_error("NTT launch failed");
      const bool small = j2 <= ntt2s_below;
      if (small ? orion_launch_ntt2s(logN, b, d_tb, inv, cs_stream[1]) : orion_launch_ntt2(logN, b, d_tb, inv, cs_stream[1]))
        throw std::runtime_error("NTT launch failed");
      HIPCHK(hipEventRecord(cs_ev[1], cs_stream[0]));
      HIPCHK(hipEventRecord(cs_ev[2], cs_stream[1]));
      HIPCHK(hipStreamWaitEvent(stream, cs_ev[1], 0));
      HIPCHK(hipStreamWaitEvent(stream, cs_ev[2], 0));
      a.jobs = j1;
      b.jobs = j2;
      log_ntt(1, a, inv);
      log_ntt(small ? 3 : 2, b, inv);
      return;
    }
    const int tail = io.jobs % n_cu;
    if (ntt_tailsplit && logN == 15 && !ci && io.jobs > n_cu && tail > 0 && tail <= ntt_tailsplit_max) {
      // the whole rounds on the one-pass kernel, the partial last round (the
      // fast float64 limbs: job order 2) on the two-pass kernels, which scale
      // with the job count instead of costing a whole limb's latency on every CU
      Scope sc(this, cat, per * io.jobs, strict * io.jobs);
      NttIO a = io;
      a.njob = io.jobs - tail;
      if (orion_launch_ntt_io(logN, a, d_tb, inv, stream)) throw std::runtime_error("NTT launch failed");
      NttIO b = io;
      Poly scratch = alloc(1, 1, tail);
      b.mid = ls(scratch, 0, 1, {0}, {0});
      b.mid_compact = 1;
      b.job0 = io.jobs - tail;
      b.njob = tail;
      const bool small = tail <= ntt2s_below;
      if (small ? orion_launch_ntt2s(logN, b, d_tb, inv, stream) : orion_launch_ntt2(logN, b, d_tb, inv, stream))
        throw std::runtime_error("NTT launch failed");
      a.jobs = a.njob;
      b.jobs = tail;
      log_ntt(1, a, inv);
      log_ntt(small ? 3 : 2, b, inv);
      return;
    }
    if (ntt_stagger > 0) {
      io.stagger = io.jobs >= ntt_stagger_min * cus() ? ntt_stagger : 0;
    }
    // algorithmic bytes per limb-transform: read + write the limb (16 N), + 8 N
    // for the epilogue's second operand (per, above)
    Scope sc(this, cat, per * io.dst.ncomp * io.dst.nlimb * io.dst.nbatch, strict * io.dst.ncomp * io.dst.nlimb * io.dst.nbatch);
    if (orion_launch_ntt_io(logN, io, d_tb, inv, stream)) throw std::runtime_error("NTT launch failed");
    log_ntt(1, io, inv);
  }
  void ntt(const LimbSet& s, bool inv) { ntt_io(nio(s, s), inv); }
  void ew(int op, const LimbSet& o, const LimbSet& a, const LimbSet& b, const std::vector<u64>* sc = nullptr) {
    std::vector<u64> s, ss;
    if (sc) {
      s = *sc;
      for (int l = 0; l < o.nlimb; ++l) ss.push_back(hm_shoup(s[l], mods[o.mod[l]]));
    }
    int nin = (op == EW_NEG || op == EW_SCALE || op == EW_ADDC || op == EW_COPY || op == EW_SPLIT24)
                  ? 1
                  : 2;
    if (op == EW_MULADD || op == EW_ADDSCALE) nin += 1;
    Scope scp(this, P_EW, 8.0 * N * o.ncomp * o.nlimb * o.nbatch * (nin + 1));
    orion_launch_ew(op, o, a, b, sc ? s.data() : nullptr, sc ? ss.data() : nullptr, d_tb, N, stream);
  }
  void ew1(int op, const LimbSet& o, const LimbSet& a, const std::vector<u64>* sc = nullptr) { ew(op, o, a, a, sc); }
  void copy(const LimbSet& o, const LimbSet& a) { ew(EW_COPY, o, a, a); }

  // -- tables ---------------------------------------------------------------------
  void setup(int logN_, const std::vector<int>& logQ, const std::vector<int>& logP, int logScale_, int h_,
             bool ci_ = false) {
    if ((int)(logQ.size() + logP.size()) > ORION_MAXMOD) throw std::runtime_error("too many moduli");
    for (int b : logQ)
      if (b > 61) throw std::runtime_error("moduli must be <= 61 bits");
    for (int b : logP)
      if (b > 61) throw std::runtime_error("moduli must be <= 61 bits");
    if (logN_ < 13 || logN_ > 16) throw std::runtime_error("logN must be 13..16 in this build");
    init_moduli(logN_, gen_moduli(logN_ + (ci_ ? 1 : 0), logQ, logP), logQ, logP, logScale_, h_, ci_);  // q = 1 mod NthRoot
  }
  // tables for explicit moduli m = [Q..., P...] (|Q| = |logQ|, |P| = |logP|)
  void init_moduli(int logN_, const std::vector<u64>& m, const std::vector<int>& logQ, const std::vector<int>& logP,
                   int logScale_, int h_, bool ci_) {
    logN = logN_;
    N = 1 << logN;
    ci = ci_;
    slots = ci ? N : N / 2;
    nthroot = (2 * (u64)N) << (ci ? 1 : 0);
    L = (int)logQ.size();
    K = (int)logP.size();
    if (K < 1) throw std::runtime_error("at least one P prime is required (hybrid key switching)");
    dnum = (L + K - 1) / K;
    logScale = logScale_;
    h = h_;
    if (L + K > ORION_MAXMOD || L + K > ORION_MAXLIMB) throw std::runtime_error("too many moduli");
    // the lazy NTT ranges (NTT_INT_CUT keeps forward values in [0, 8q)) and
    // lt_bsgs's 8-product Barrett (barrett_8q2, bar_k <= 60 for x < 8 q^2)
    // hold only for moduli below 2^61 (ntt_arith.h)
    for (u64 q : m)
      if (q >= (1ull << 61) || q < 3 || !(q & 1)) throw std::runtime_error("moduli must be odd and below 2^61");
    mods = m;
    logQ_bits = logQ;
    logP_bits = logP;
    if (!stream) {
      HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
      own_stream = true;
    }
    orion_ntt_init();
    memset(&host_tb, 0, sizeof(host_tb));
    for (int m = 0; m < L + K; ++m) build_mod_tables(m);
    HIPCHK(hipMalloc(&d_tb, sizeof(DeviceTables)));
    HIPCHK(hipMemcpy(d_tb, &host_tb, sizeof(DeviceTables), hipMemcpyHostToDevice));
    for (int inv = 0; inv < 2; ++inv) {
      const std::vector<Cplx> tw = special_fft_twiddles(logN + (ci ? 1 : 0), inv != 0);  // slots = 2^(that - 1)
      void* d;
      HIPCHK(hipMalloc(&d, tw.size() * sizeof(double2)));
      HIPCHK(hipMemcpy(d, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice));
      static_bufs.push_back(d);
      (inv ? tw_inv : tw_fwd) = (double2*)d;
    }
    // the blocking table copies above ran on the legacy NULL stream, which the
    // library stream does not wait for: drain the device before any kernel
    // reads a twiddle or constant table
    HIPCHK(hipDeviceSynchronize());
    memset(&enc_sampler, 0, sizeof(enc_sampler));
    gauss_cdt(3.2, ORION_GAUSS_BOUND, enc_sampler.cdt);
  }
  std::vector<int> logQ_bits, logP_bits;
  // per-modulus constants and NTT twiddle tables of QP index m (host_tb; device copy by the caller)
  void build_mod_tables(int m) {
    std::vector<ulonglong2> fw(N), iv(N);
    {
      const u64 q = mods[m];
      ModConst& mc = host_tb.mc[m];
      mc.q = q;
      mc.bar_k = 64 - __builtin_clzll(q);
      mc.bar_mu = (u64)(((u128)1 << (2 * mc.bar_k)) / q);
      mc.bar_mu2 = (u64)(((u128)1 << (2 * mc.bar_k + 2)) / q);
      mc.bar_mu8 = mc.bar_k <= 52 ? (u64)(((u128)1 << (2 * mc.bar_k + 8)) / q) : 0;
      mc.bar_mu3 = mc.bar_k <= 60 ? (u64)(((u128)1 << (2 * mc.bar_k + 3)) / q) : 0;
      // CI: the unfold's 1/2 rides on the inverse's final scaling, (2N)^-1
      mc.ninv = hm_invmod((u64)N << (ci ? 1 : 0), q);
      mc.ninv_s = hm_shoup(mc.ninv, q);
      const u64 g = primitive_root(q);
      const u64 psi = hm_powmod(g, (q - 1) / nthroot, q);  // primitive NthRoot-th root
      const u64 psii = hm_invmod(psi, q);
      // twiddles of the degree-M negacyclic NTT, M = NthRoot / 2, bit-reversed
      const int logM = logN + (ci ? 1 : 0), M = 1 << logM;
      std::vector<u64> tf(M), ti(M);
      u64 a = 1, b = 1;
      for (int j = 0; j < M; ++j) {
        const u64 r = hm_bitrev(j, logM);
        tf[r] = a;
        ti[r] = b;
        a = hm_mulmod(a, psi, q);
        b = hm_mulmod(b, psii, q);
      }
      // CI: after the fold, the N-point stage with m groups is the degree-2N
      // NTT's stage with 2m groups on its first half: twiddle m + i -> 2m + i
      // (oracle_new_ring)
      for (int k = 0; k < N; ++k) {
        int mm = 1;
        while (2 * mm <= k) mm <<= 1;
        const int src = ci ? (k ? k + mm : 0) : k;
        fw[k] = make_ulonglong2(tf[src], hm_shoup(tf[src], q));
        iv[k] = make_ulonglong2(ti[src], hm_shoup(ti[src], q));
      }
      mc.wl = hm_mulmod(iv[1].x, mc.ninv, q);
      mc.wl_s = hm_shoup(mc.wl, q);
      mc.ciw = ci ? tf[1] : 0;  // psi^N
      mc.ciw_s = ci ? hm_shoup(tf[1], q) : 0;
      // float64-path constants and centered twiddles for small moduli
      mc.f64 = mc.bar_k <= ORION_F64_BITS ? 1 : 0;
      mc.qd = (double)q;
      mc.qinv_d = 1.0 / (double)q;
      mc.ninv_d = (double)(mc.ninv > q / 2 ? (long long)mc.ninv - (long long)q : (long long)mc.ninv);
      mc.wl_d = (double)(mc.wl > q / 2 ? (long long)mc.wl - (long long)q : (long long)mc.wl);
      if (mc.f64) {
        std::vector<double> fd(N), id(N);
        for (int j = 0; j < N; ++j) {
          const u64 a1 = fw[j].x, b1 = iv[j].x;
          fd[j] = (double)(a1 > q / 2 ? (long long)a1 - (long long)q : (long long)a1);
          id[j] = (double)(b1 > q / 2 ? (long long)b1 - (long long)q : (long long)b1);
        }
        void *dfd, *did;
        HIPCHK(hipMalloc(&dfd, N * sizeof(double)));
        HIPCHK(hipMalloc(&did, N * sizeof(double)));
        HIPCHK(hipMemcpy(dfd, fd.data(), N * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(did, id.data(), N * sizeof(double), hipMemcpyHostToDevice));
        static_bufs.push_back(dfd);
        static_bufs.push_back(did);
        host_tb.fwd_d[m] = (const double*)dfd;
        host_tb.inv_d[m] = (const double*)did;
      }
      void *dfw, *div;
      HIPCHK(hipMalloc(&dfw, N * sizeof(ulonglong2)));
      HIPCHK(hipMalloc(&div, N * sizeof(ulonglong2)));
      HIPCHK(hipMemcpy(dfw, fw.data(), N * sizeof(ulonglong2), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(div, iv.data(), N * sizeof(ulonglong2), hipMemcpyHostToDevice));
      static_bufs.push_back(dfw);
      static_bufs.push_back(div);
      host_tb.fwd[m] = (const ulonglong2*)dfw;
      host_tb.inv[m] = (const ulonglong2*)div;
    }
  }

  // secret key coefficients (ternary) from its first limb
  std::vector<int64_t> secret_coeffs() {
    Poly t = alloc(1, 1, 1);
    ntt_io(nio(ls(t, 0, 1, {0}, {0}), ls(sk, 0, 1, {0}, {0})), true);
    std::vector<u64> host;
    download(t, host);
    std::vector<int64_t> s(N);
    const u64 q0 = mods[0];
    for (int i = 0; i < N; ++i) s[i] = host[i] > q0 / 2 ? -(int64_t)(q0 - host[i]) : (int64_t)host[i];
    return s;
  }
  // encryption randomness: ChaCha20 key from the seed, encryption index 0
  void seed_encryption(u64 seed) {
    enc_key_from_seed(seed, enc_sampler.key);
    enc_sampler.enc = 0;
  }

  u64 prod_mod(const std::vector<int>& src, int skip, u64 t) const {
    u64 r = 1 % t;
    for (int i = 0; i < (int)src.size(); ++i)
      if (i != skip) r = hm_mulmod(r, mods[src[i]] % t, t);
    return r;
  }

  // how a target's sum is formed (common.h BextTarget): every bound is checked
  // with the actual moduli, so each column and the final value fit their words
  // (the terms: y_i < s_i times qh_i < t, and v <= ns times nS < t)
  // 0: BEXT_WT / BEXT_NT off (timing switch)
  int bext_modes = getenv("ORION_BEXT_MODES") ? atoi(getenv("ORION_BEXT_MODES")) : 1;
  int bext_mode(const std::vector<int>& src, int ns, u64 t) const {
    const u128 M30 = (1u << 30) - 1, T1 = t - 1;
    u128 ssum = ns;  // sum (s_i - 1) + ns
    bool src32 = true, src62 = true;
    for (int i = 0; i < ns; ++i) {
      const u64 si = mods[src[i]];
      ssum += si - 1;
      src32 = src32 && si < (1ull << 32);
      src62 = src62 && si < (1ull << 62);
    }
    const u128 two64 = (u128)1 << 64;
    if (src32 && t < (1ull << 32) && (ssum + 1) * t < ((u128)1 << 63)) return BEXT_NARROW;
    if (!bext_modes) return BEXT_LAZY;
    if (ns >= 3 && src32 && t >= (1ull << 32) && t < (1ull << 61) && ssum * M30 < two64 &&
        ssum * T1 < (u128)4 * t * t)
      return BEXT_WT;
    // (columns: ns + 1 terms of a 30-bit piece times t - 1; the whole sum below
    // 2^96, so the folded high word is below 2^32)
    if (ns >= 4 && src62 && t < (1ull << 31) && (u128)(ns + 1) * M30 * T1 < two64 && ssum * T1 < ((u128)1 << 96))
      return BEXT_NT;
    return BEXT_LAZY;
  }

  // centered: a gadget digit (Lattigo DecomposeAndSplit extends a one-prime
  // digit from its centered representative; ModDown's ModUpExact does not)
  BasisExtTable* make_betab(const std::vector<int>& src, const std::vector<int>& dst, bool centered = false) {
    no_capture("a basis extension table");
    BasisExtTable T;
    memset(&T, 0, sizeof(T));
    T.ns = (int)src.size();
    T.nt = (int)dst.size();
    T.centered = centered && T.ns == 1 ? 1 : 0;
    T.chalf = mods[src[0]] >> 1;
    if (T.ns > ORION_MAXSRC || T.nt > ORION_MAXLIMB) throw std::runtime_error("basis extension too large");
    for (int i = 0; i < T.ns; ++i) {
      const u64 si = mods[src[i]];
      T.src_mod[i] = src[i];
      T.sq[i] = si;
      T.qhatinv[i] = hm_invmod(prod_mod(src, i, si), si);
      T.qhatinv_s[i] = hm_shoup(T.qhatinv[i], si);
      T.qf[i] = (double)si;
      T.qinv_f[i] = 1.0 / T.qf[i];
    }
    for (int t = 0; t < T.nt; ++t) {
      const u64 tm = mods[dst[t]];
      BextTarget& R = T.tgt[t];
      T.dst_mod[t] = dst[t];
      R.q = tm;
      const u64 S = prod_mod(src, -1, tm);
      for (int i = 0; i < T.ns; ++i) {
        R.qh[i] = prod_mod(src, i, tm);
        R.qhs[i] = hm_shoup(R.qh[i], tm);
      }
      R.nS = S ? tm - S : 0;
      R.nSs = hm_shoup(R.nS, tm);
      for (int v = 0; v < 3; ++v) R.vS[v] = hm_mulmod((u64)v, R.nS, tm);
      R.qd = (double)tm;
      R.tinv = 1.0 / (double)tm;
      R.tinv32 = std::ldexp(R.tinv, 32);
      R.k = 64 - __builtin_clzll(tm);
      R.mu2 = R.k <= 61 ? (u64)(((u128)1 << (2 * R.k + 2)) / tm) : 0;
      R.c64 = (u64)(((u128)1 << 64) % tm);
      auto pieces = [](u64 x, u32& a, u32& b, u32& c) {
        a = (u32)(x & 0x3fffffffu), b = (u32)((x >> 30) & 0x3fffffffu), c = (u32)(x >> 60);
      };
      for (int i = 0; i < T.ns; ++i) pieces(R.qh[i], R.h0[i], R.h1[i], R.h2[i]);
      pieces(R.nS, R.n0, R.n1, R.n2);
      R.mode = T.centered ? BEXT_LAZY : bext_mode(src, T.ns, tm);
    }
    BasisExtTable* d;
    HIPCHK(hipMalloc(&d, sizeof(T)));
    h2d(d, &T, sizeof(T));
    return d;
  }
  // ModUp of digit i at level: sources Q[lo,hi), targets = rest of QP in QP-position order
  BasisExtTable* modup_tab(int level, int digit, std::vector<int>& tpos) {
    auto key = std::make_pair(level, digit);
    auto it = betab.find(key);
    if (it != betab.end()) {
      tpos = betab_pos[key];
      return it->second;
    }
    const int lo = digit * K, hi = std::min((digit + 1) * K, level + 1);
    std::vector<int> src = iota(lo, hi), dst;
    tpos.clear();
    for (int j = 0; j <= level + K; ++j) {
      if (j >= lo && j < hi) continue;
      tpos.push_back(j);
      dst.push_back(qp_mod(level, j));
    }
    BasisExtTable* d = make_betab(src, dst, true);
    betab[key] = d;
    betab_pos[key] = tpos;
    return d;
  }
  // copies of the digits' ModUp tables in one array, so that modup_all_kernel
  // indexes them off a kernel argument (noalias: wave-uniform table reads
  // become scalar loads; through an array of pointers they were vector loads)
  const BasisExtTable* modup_tabs(int level) {
    auto it = modup_arr.find(level);
    if (it != modup_arr.end()) return it->second;
    no_capture("the ModUp table array");
    const int beta = (level + 1 + K - 1) / K;
    BasisExtTable* d;
    HIPCHK(hipMalloc(&d, sizeof(BasisExtTable) * beta));
    std::vector<int> tpos;
    for (int i = 0; i < beta; ++i)
      HIPCHK(hipMemcpyAsync(d + i, modup_tab(level, i, tpos), sizeof(BasisExtTable), hipMemcpyDeviceToDevice,
                             stream));
    HIPCHK(hipStreamSynchronize(stream));
    modup_arr[level] = d;
    return d;
  }
  BasisExtTable* moddown_tab(int level) {
    auto key = std::make_pair(level, -1);
    auto it = betab.find(key);
    if (it != betab.end()) return it->second;
    std::vector<int> src;
    for (int k = 0; k < K; ++k) src.push_back(L + k);
    BasisExtTable* d = make_betab(src, iota(0, level + 1));
    betab[key] = d;
    return d;
  }

  u64 galois_element(int k) const {
    return hm_powmod(5, (u64)(long long)k & (nthroot - 1), nthroot);
  }
  const u32* aut_index(u64 g) {
    auto it = autidx.find(g);
    if (it != autidx.end()) return it->second;
    no_capture("an automorphism index table");
    // CI: the index over the degree-2N NTT; the ring keeps its first half,
    // which every g = 5^k (= 1 mod 4) maps onto itself
    std::vector<u32> idx(N);
    const int logM = logN + (ci ? 1 : 0);
    const u64 mask = nthroot - 1;
    for (int j = 0; j < N; ++j) {
      const u64 t1 = 2 * hm_bitrev(j, logM) + 1;
      const u64 t2 = (((g * t1) & mask) - 1) >> 1;
      idx[j] = (u32)hm_bitrev(t2, logM);
      if (idx[j] >= (u32)N) throw std::runtime_error("Galois element does not act on the ring");
    }
    u32* d;
    HIPCHK(hipMalloc(&d, N * sizeof(u32)));
    h2d(d, idx.data(), N * sizeof(u32));
    autidx[g] = d;
    return d;
  }
  void automorph(const LimbSet& o, const LimbSet& a, u64 g, bool acc) {
    const u32* idx = aut_index(g);
    Scope sc(this, P_AUT, 8.0 * N * o.ncomp * o.nlimb * o.nbatch * (acc ? 3 : 2));
    orion_launch_automorph(o, a, idx, d_tb, N, acc ? 1 : 0, stream);
  }

  // -- upload of host residues (coefficient domain) + NTT -------------------------------
  void upload(const Poly& P, const std::vector<u64>& host) {
    no_capture("a host upload");
    HIPCHK(hipMemcpyAsync(P.ptr(), host.data(), host.size() * sizeof(u64), hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  void download(const Poly& P, std::vector<u64>& host) {
    no_capture("a host download");
    host.resize((size_t)P.ncomp * P.nlimb * P.B * N);
    HIPCHK(hipMemcpyAsync(host.data(), P.ptr(), host.size() * sizeof(u64), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  // small signed coefficients -> residues for moduli md, into host[l*N + n] of a [nl][N] block
  void small_residues(const std::vector<int64_t>& v, const std::vector<int>& md, u64* out) const {
    for (size_t l = 0; l < md.size(); ++l) {
      const u64 q = mods[md[l]];
      for (int n = 0; n < N; ++n) {
        const int64_t x = v[n];
        out[l * N + n] = x >= 0 ? (u64)x % q : (q - ((u64)(-x) % q)) % q;
      }
    }
  }
  std::vector<int64_t> sample_gauss() {
    std::vector<int64_t> e(N);
    for (auto& x : e) x = prng.gaussian(3.2, 19.2);
    return e;
  }
  std::vector<int64_t> sample_ternary_h(int hw) {
    std::vector<int64_t> s(N, 0);
    std::vector<int> perm(N);
    for (int i = 0; i < N; ++i) perm[i] = i;
    hw = std::min(hw, N);
    for (int i = 0; i < hw; ++i) {
      const int j = i + (int)(prng.next() % (u64)(N - i));
      std::swap(perm[i], perm[j]);
      s[perm[i]] = (prng.next() & 1) ? 1 : -1;
    }
    return s;
  }
  std::vector<u64> qp_mod_list() const {
    std::vector<u64> v;
    for (int j = 0; j < L + K; ++j) v.push_back(mods[j]);
    return v;
  }

  // ---------------------------------------------------------------------------
  // keys
  // ---------------------------------------------------------------------------
  void gen_secret() { import_secret(sample_ternary_h(h)); }
  // a secret with these (ternary) coefficients, expanded over QP (NTT domain)
  Poly secret_poly(const std::vector<int64_t>& s) {
    Poly p = alloc(1, L + K, 1);
    std::vector<u64> host((size_t)(L + K) * N);
    small_residues(s, iota(0, L + K), host.data());
    upload(p, host);
    ntt(ls(p, 0, 1, iota(0, L + K), iota(0, L + K)), false);
    return p;
  }
  void import_secret(const std::vector<int64_t>& s) {
    sk = secret_poly(s);
    have_sk = true;
  }
  // another context's keys (same chain), shared: the key polys are the same
  // device buffers (read-only once made), the loaded keys' host copies the
  // same host arrays
  void adopt_keys(const Context& o) {
    if (o.mods != mods) throw std::runtime_error("pipeline context: another modulus chain");
    HIPCHK(hipStreamSynchronize(o.stream));
    if (o.have_sk) sk = o.sk, have_sk = true;
    if (o.have_pk) pk = o.pk, have_pk = true;
    if (o.have_rlk) rlk = o.rlk, have_rlk = true;
    gks = o.gks;
    key_hint = o.key_hint;
    gk_host = o.gk_host;
  }
  LimbSet full(const Poly& P, int c0, int nc) const { return ls(P, c0, nc, iota(0, L + K), iota(0, L + K)); }

  void gen_public() {
    if (!have_sk) throw std::runtime_error("secret key not generated");
    pk = alloc(2, L + K, 1);
    std::vector<u64> a((size_t)(L + K) * N), e((size_t)(L + K) * N);
    for (int m = 0; m < L + K; ++m)
      for (int n = 0; n < N; ++n) a[(size_t)m * N + n] = prng.uniform(mods[m]);
    small_residues(sample_gauss(), iota(0, L + K), e.data());
    Poly tmp = alloc(1, L + K, 1);
    HIPCHK(hipMemcpyAsync(pk.ptr() + pk.comp_stride(), a.data(), a.size() * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(pk.ptr(), e.data(), e.size() * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
    ntt(full(pk, 0, 1), false);
    ew(EW_MUL, full(tmp, 0, 1), full(pk, 1, 1), full(sk, 0, 1));
    ew(EW_SUB, full(pk, 0, 1), full(pk, 0, 1), full(tmp, 0, 1));
    have_pk = true;
  }

  // QP moduli of a key made for `level`: q_0..q_level, then p_0..p_{K-1}
  std::vector<int> key_mods(int level) const {
    std::vector<int> v = iota(0, level + 1);
    for (int k = 0; k < K; ++k) v.push_back(L + k);
    return v;
  }
  // evaluation key switching s_in -> s_out for ciphertexts up to `level`,
  // layout [beta][2][level+1+K][N] (beta = ceil((level+1)/K) digits); a
  // full-chain key (level L - 1) is [dnum][2][L+K][N]
  Poly gen_evk(const Poly& s_in, const Poly& s_out, int level) {
    no_capture("evaluation key generation");
    const int beta = (level + 1 + K - 1) / K, nl = level + 1 + K;
    const std::vector<int> md = key_mods(level), kp = iota(0, nl);
    Poly k = alloc(2 * beta, nl, 1);
    Poly tmp = alloc(1, nl, 1);
    std::vector<u64> a((size_t)nl * N), e((size_t)nl * N);
    for (int i = 0; i < beta; ++i) {
      for (int x = 0; x < nl; ++x)
        for (int n = 0; n < N; ++n) a[(size_t)x * N + n] = prng.uniform(mods[md[x]]);
      small_residues(sample_gauss(), md, e.data());
      HIPCHK(hipMemcpyAsync(k.ptr() + (2 * i + 1) * k.comp_stride(), a.data(), a.size() * 8,
                            hipMemcpyHostToDevice, stream));
      HIPCHK(hipMemcpyAsync(k.ptr() + (2 * i) * k.comp_stride(), e.data(), e.size() * 8, hipMemcpyHostToDevice,
                            stream));
      HIPCHK(hipStreamSynchronize(stream));
      const LimbSet kb = ls(k, 2 * i, 1, kp, md), ka = ls(k, 2 * i + 1, 1, kp, md), lt = ls(tmp, 0, 1, kp, md);
      ntt(kb, false);
      ew(EW_MUL, lt, ka, ls(s_out, 0, 1, md, md));
      ew(EW_SUB, kb, kb, lt);
      // + P * s_in on the Q limbs of digit i
      const int lo = i * K, hi = std::min((i + 1) * K, level + 1);
      std::vector<int> dl = iota(lo, hi);
      std::vector<u64> pm;
      for (int j : dl) {
        u64 P = 1;
        for (int kk = 0; kk < K; ++kk) P = hm_mulmod(P, mods[L + kk] % mods[j], mods[j]);
        pm.push_back(P);
      }
      ew(EW_ADDSCALE, ls(k, 2 * i, 1, dl, dl), ls(s_in, 0, 1, dl, dl), ls(s_in, 0, 1, dl, dl), &pm);
    }
    return k;
  }
  void gen_relin() {
    if (!have_sk) throw std::runtime_error("secret key not generated");
    Poly s2 = alloc(1, L + K, 1);
    ew(EW_MUL, full(s2, 0, 1), full(sk, 0, 1), full(sk, 0, 1));
    rlk = gen_evk(s2, sk, L - 1);
    have_rlk = true;
  }
  // LoadRotationKey's whole keys, for the ones it cut on the device
  struct HostKey {
    int level = 0;
    std::shared_ptr<const std::vector<u64>> words;  // [digit][2][level+1+K][N] (shared with the pipelines)
  };
  std::map<u64, HostKey> gk_host;
  int hinted_level(u64 g) const {
    auto it = key_hint.find(g);
    return it == key_hint.end() ? L - 1 : it->second;
  }
  // the Galois key of g, made for at least `level` (a key made for a lower
  // level is replaced by one for this level)
  void gen_galois(u64 g, int level) {
    auto have = gks.find(g);
    if (have != gks.end() && have->second.level >= level) return;
    // a pipeline's keys are the scheme's: a key it lacks (made, loaded or
    // raised to a higher level after the pipeline was created) is made by the
    // scheme's context, with the scheme's randomness, and shared, so every
    // context switches with the same key and a pipeline's output equals the
    // scheme's bit for bit
    Context* s = scheme_ctx();
    if (index > 0 && s && s != this) {
      no_capture("taking a Galois key from the scheme");
      std::lock_guard<std::recursive_mutex> lk(s->mu);  // (a pipeline may wait on the scheme: index order)
      s->gen_galois(g, level);
      HIPCHK(hipStreamSynchronize(s->stream));
      // the replaced key's buffer may return to the scheme's pool once this
      // context lets go of it: this stream is done reading it first
      if (have != gks.end()) HIPCHK(hipStreamSynchronize(stream));
      gks[g] = s->gks.at(g);
      return;
    }
    auto hk = gk_host.find(g);
    if (hk != gk_host.end() && hk->second.level >= level) {  // a loaded key, cut at load: the whole key
      no_capture("uploading a loaded rotation key past its cut level");
      const int kl = hk->second.level, kb = (kl + 1 + K - 1) / K;
      Poly k = alloc(2 * kb, kl + 1 + K, 1);
      upload(k, *hk->second.words);
      gks[g] = EvKey{k, kl};
      gk_host.erase(hk);
      return;
    }
    if (!have_sk)
      throw std::runtime_error(have == gks.end() ? "secret key not generated"
                                                 : "galois key " + std::to_string(g) + " covers level " +
                                                       std::to_string(have->second.level) + " < " +
                                                       std::to_string(level) +
                                                       " and there is no secret key (LoadRotationKey keeps a key "
                                                       "over the highest level of the linear transforms that exist "
                                                       "when it is loaded: load keys after creating the transforms "
                                                       "and before any higher-level rotation)");
    const u64 ginv = galois_inverse(g);
    Poly s_out = alloc(1, L + K, 1);
    automorph(full(s_out, 0, 1), full(sk, 0, 1), ginv, false);
    gks[g] = EvKey{gen_evk(sk, s_out, level), level};
  }
  const EvKey& galois_key(u64 g, int level) {
    gen_galois(g, level);  // Lattigo AddRotationKey semantics: generate on first use
    return gks.at(g);
  }

  // ---------------------------------------------------------------------------
  // key switching building blocks
  // ---------------------------------------------------------------------------
  // sub-range [first, first+count) of a LimbSet's limbs
  static LimbSet limbs(const LimbSet& x, int first, int count) {
    LimbSet s = x;
    s.nlimb = count;
    for (int i = 0; i < count; ++i) {
      s.pos[i] = x.pos[first + i];
      s.mod[i] = x.mod[first + i];
    }
    return s;
  }
  // decompose c.ncomp Q polys (limbs 0..level of c) into beta digits each,
  // extended to QP and in the NTT domain.  D layout [comp][digit][QP][B], QP
  // positions at lvl_alloc = level.  Digit i's own Q limbs (l / K == i) equal
  // c's and are not written: every consumer (ks_mac, lt_bsgs, lt_giant) reads
  // them from c.
  // want_cols_only: if the decomposition takes the fused latency path, its
  // forward NTT stops after the columns pass (the caller's gadget product runs
  // the rows pass, ks_mac_full_kernel); *cols_only tells whether it did
  Poly decompose(const LimbSet& c, int level, int B, bool want_cols_only = false, bool* cols_only = nullptr) {
    if (cols_only) *cols_only = false;
    const int nc = c.ncomp;
    const int beta = (level + 1 + K - 1) / K;
    const int nqp = level + 1 + K;
    Poly cinv = alloc(nc, level + 1, B);
    const NttIO iio = nio(lsq(cinv, 0, nc, level), c);  // out-of-place INTT
    Poly D = alloc(nc * beta, nqp, B);
    if (nc * B * (nqp - K) < modup_merge && nqp <= ORION_MAXLIMB) {
      // small decomposition: every digit's ModUp in one launch (own limbs not
      // written), then one NTT over every digit's target limbs: limb (digit i,
      // QP position j) of comp c sits at comp c, position i*nqp + j of a
      // LimbSet whose comp stride spans the beta digits
      std::vector<int> md;
      for (int j = 0; j < nqp; ++j) md.push_back(qp_mod(level, j));
      LimbSet Dl = ls(D, 0, nc * beta, iota(0, nqp), md);
      LimbSet in = ls(cinv, 0, nc, iota(0, level + 1), iota(0, level + 1));
      std::vector<int> tpos, tmod;
      for (int i = 0; i < beta; ++i)
        for (int j = 0; j < nqp; ++j)
          if (!(j >= i * K && j < std::min((i + 1) * K, level + 1))) tpos.push_back(i * nqp + j), tmod.push_back(md[j]);
      const bool tset = beta * nqp <= 256 && (int)tpos.size() <= ORION_MAXLIMB;
      if (tset && fuse_bext(nc * B * (int)tpos.size(), K, NTT_EPI_STORE)) {
        // every digit's extension formed in the prologue of one NTT over the
        // target limbs (no modup_all launch, no round trip through HBM)
        LimbSet T = ls(D, 0, nc, tpos, tmod);
        T.comp_stride = (long long)beta * D.comp_stride();
        NttIO io = nio(T, in);
        io.pro = NTT_PRO_BEXT;
        io.bx = modup_tabs(level);
        for (int i = 0; i < beta; ++i) io.bx_s0[i] = (unsigned char)(i * K);
        double srcs = 0;
        for (size_t l = 0; l < tpos.size(); ++l) {
          const int i = tpos[l] / nqp, j = tpos[l] % nqp, lo = i * K, ns = std::min(K, level + 1 - lo);
          io.bx_tab[l] = (unsigned char)i;
          io.bx_t[l] = (unsigned char)(j < lo ? j : j - ns);
          srcs += ns;
        }
        if (want_cols_only && ifuse_ok(iio, io, K)) {
          io.cols_only = 1;
          if (cols_only) *cols_only = true;
        }
        intt_then_fwd(iio, io, K, srcs / (double)tpos.size());
        return D;
      }
      ntt_io(iio, true);
      {
        Scope sc(this, P_BEXT, 8.0 * N * B * nc * (level + 1 + beta * nqp - (level + 1)));
        if (orion_launch_modup_all(Dl, in, modup_tabs(level), beta, K, nqp, d_tb, N, stream))
          throw std::runtime_error("modup_all: bad launch shape");
      }
      if (tset) {
        LimbSet T = ls(D, 0, nc, tpos, tmod);
        T.comp_stride = (long long)beta * D.comp_stride();
        ntt(T, false);
      } else {
        ntt(Dl, false);  // (own limbs transformed too; their contents are unused)
      }
      return D;
    }
    ntt_io(iio, true);
    const long long dstride = (long long)beta * D.comp_stride();
    for (int i = 0; i < beta; ++i) {
      const int lo = i * K, hi = std::min((i + 1) * K, level + 1);
      std::vector<int> tpos;
      BasisExtTable* T = modup_tab(level, i, tpos);
      std::vector<int> tmod;
      for (int p : tpos) tmod.push_back(qp_mod(level, p));
      LimbSet in = ls(cinv, 0, nc, iota(lo, hi), iota(lo, hi));
      LimbSet out = ls(D, i, nc, tpos, tmod);
      out.comp_stride = dstride;
      if (fuse_bext(nc * B * out.nlimb, hi - lo, NTT_EPI_STORE)) {  // the extension formed in the NTT's prologue
        NttIO io = nio(out, in);
        io.pro = NTT_PRO_BEXT;
        io.bx = T;
        for (int t = 0; t < out.nlimb; ++t) io.bx_tab[t] = 0, io.bx_t[t] = (unsigned char)t;
        io.bx_s0[0] = 0;
        ntt_io(io, false, hi - lo);
        continue;
      }
      // ModUp as its own kernel (the ORION_BEXT_FUSE=0 path, and digits of more
      // than 2 limbs): y_i and the float64 quotient are shared by every target
      {
        Scope sc(this, P_BEXT, 8.0 * N * B * nc * (in.nlimb + out.nlimb));
        if (orion_launch_basis_ext(out, in, T, d_tb, N, stream))
          throw std::runtime_error("basis_ext: unsupported source count");
      }
      ntt(out, false);
    }
    return D;  // the own Q limbs of each digit are left unset: consumers read them from c

  }
  // grouped gadget products: out_g (comps 0/1 at o.p + g*out_gstride) =
  //   [add0_g on comp 0] + sum_i D_g,i * keys[g]_i,   D_g at d.p + g*d_gstride,
  // own Q limbs of each digit read from own (group stride own_gstride)
  void mac_groups(const LimbSet& o, long long out_gstride, const LimbSet& d, long long d_gstride,
                  const LimbSet& own, long long own_gstride, const std::vector<const u64*>& keys,
                  const std::vector<int>& klvl, int beta, const u64* add0 = nullptr, long long add_gstride = 0,
                  int add_nq = 0, const u64* add1 = nullptr, int rows_from = 0, bool fwd_rows = false) {
    const int G = (int)keys.size();
    for (int g0 = 0; g0 < G; g0 += ORION_MAXGROUP) {
      const int ng = std::min(ORION_MAXGROUP, G - g0);
      MacGroups mg;
      memset(&mg, 0, sizeof(mg));
      for (int g = 0; g < ng; ++g) mg.key[g] = keys[g0 + g], mg.klvl[g] = klvl[g0 + g];
      mg.L = L;
      mg.out_gstride = out_gstride;
      mg.d_gstride = d_gstride;
      mg.add_gstride = add_gstride;
      mg.own_gstride = own_gstride;
      mg.K = K;
      mg.add0 = add0 ? add0 + g0 * add_gstride : nullptr;
      mg.add1 = add1 ? add1 + g0 * add_gstride : nullptr;
      mg.add_nq = add0 ? add_nq : 0;
      mg.rows_from = rows_from;
      mg.logN = logN;
      mg.fwd_rows = (fwd_rows && rows_from > 0) ? 1 : 0;
      if (fwd_rows && rows_from == 0) throw std::runtime_error("mac_groups: forward rows without the ModDown rows pass");
      for (int j = 0; j < mg.add_nq; ++j) {  // P mod q_j: ModDown(u + P*a) = ModDown(u) + a exactly
        u64 P = 1;
        for (int k = 0; k < K; ++k) P = hm_mulmod(P, mods[L + k] % mods[o.mod[j]], mods[o.mod[j]]);
        mg.add_s[j] = P;
        mg.add_ss[j] = hm_shoup(P, mods[o.mod[j]]);
      }
      LimbSet oo = o, dd = d, ow = own;
      oo.p += g0 * out_gstride;
      dd.p += g0 * d_gstride;
      ow.p += g0 * own_gstride;
      const double rows = (double)o.nlimb * o.nbatch;
      const double dreads = d_gstride ? rows * ng * beta : rows * beta;
      const double adds = add0 ? (add_nq ? (add1 ? 2.0 : 1.0) * add_nq / o.nlimb : 1.0) : 0.0;
      Scope sc(this, P_MAC, 8.0 * N * (dreads + rows * ng * (2 + adds) + 2.0 * beta * ng * o.nlimb));
      if (orion_launch_ks_mac(oo, dd, ow, mg, ng, beta, d_tb, N, stream))
        throw std::runtime_error("ks_mac launch failed");
    }
  }
  // whether the forward NTT of jobs limb-transforms with prologue pro runs on
  // a kernel with the automorphism-scatter epilogue (NTT_EPI_SUBSCALE_AUT):
  // the one-pass kernel with the load prologue, or the radix-4 latency kernels
  bool aut_epi_ok(int jobs, int pro) {
    if (ci || ntt_tailsplit) return false;
    if (!two_pass(jobs, false, pro, NTT_EPI_SUBSCALE_AUT, false)) return logN <= 15 && pro == NTT_PRO_LOAD;
    if (md_force || jobs <= ntt2s_below) return NTT2S_R4;
    return pro == NTT_PRO_LOAD && ntt2_tail_aut;  // the large two-pass kernels (ntt2.hip), load prologue
  }
  u64 galois_inverse(u64 g) const {
    const u64 M = nthroot;
    u64 ginv = hm_powmod(g, M / 2 - 1, M);  // g^-1 mod NthRoot (the group order divides M/2)
    if ((g * ginv) % M != 1) {
      for (ginv = 1; ginv < M; ginv += 2)
        if ((g * ginv) % M == 1) break;
    }
    return ginv;
  }
  // x: x.ncomp polys, QP limbs in the order [Q 0..level][P 0..K-1] (any strides);
  // out = (x_Q - ModUp(INTT(x_P))) * P^-1.  Clobbers x's P limbs.  aut_g != 0:
  // out = sigma_g of that (a rotation's NTT-domain automorphism), applied in
  // the final NTT's store when its kernel can scatter, else by automorph();
  // aut_acc: out += sigma_g(...) instead
  // whether moddown(x, level, out, aut_g) runs its P limbs' INTT as the fused
  // latency path, so that the gadget product before it may store those limbs
  // after the INTT's rows pass (keyswitch, ks_mac_rows_kernel)
  bool moddown_rows_fusable(const LimbSet& x, int level, const LimbSet& out, u64 aut_g, bool aut_acc) {
    if (!mac_rows || (logN != 15 && logN != 16) || !NTT2S_R4) return false;
    MdForce mf(this, aut_g != 0);
    const int nc = x.ncomp, B = x.nbatch, jobs = nc * B * (level + 1);
    if (!fuse_bext(jobs, K, NTT_EPI_SUBSCALE)) return false;
    const bool scatter = aut_g && ntt_aut_fuse && aut_epi_ok(jobs, NTT_PRO_BEXT);
    if (aut_g && !scatter) return false;
    LimbSet xp = limbs(x, level + 1, K);
    NttIO io = nio(out, xp);
    io.pro = NTT_PRO_BEXT;
    io.epi = !scatter ? NTT_EPI_SUBSCALE : aut_acc ? NTT_EPI_SUBSCALE_AUT_ACC : NTT_EPI_SUBSCALE_AUT;
    io.ex = limbs(x, 0, level + 1);
    return ifuse_ok(nio(xp, xp), io, K);
  }
  // 1: keyswitch's gadget product stores the P limbs through the ModDown
  // INTT's rows pass when the ModDown takes the fused latency path
  int mac_rows = getenv("ORION_MAC_ROWS") ? atoi(getenv("ORION_MAC_ROWS")) : 1;
  // 1: ... and runs the decomposition NTT's forward rows pass itself
  int mac_fwd_rows = getenv("ORION_MAC_FWD_ROWS") ? atoi(getenv("ORION_MAC_FWD_ROWS")) : 1;
  // 1: lt_bsgs / lt_giant take their workgroups in XCD-aware order (every
  // coefficient block's diagonals and keys read into one XCD's L2)
  int lt_xcd = getenv("ORION_LT_XCD") ? atoi(getenv("ORION_LT_XCD")) : 1;
  void moddown(const LimbSet& x, int level, const LimbSet& out, u64 aut_g = 0, bool aut_acc = false,
               bool rows_done = false) {
    MdForce mf(this, aut_g != 0);
    const int nc = x.ncomp, B = x.nbatch, jobs = nc * B * (level + 1);
    LimbSet xp = limbs(x, level + 1, K);
    const bool fused = fuse_bext(jobs, K, NTT_EPI_SUBSCALE);
    const bool scatter = aut_g && ntt_aut_fuse && aut_epi_ok(jobs, fused ? NTT_PRO_BEXT : NTT_PRO_LOAD);
    Poly tmp;
    LimbSet dst = out;
    if (aut_g && !scatter) {  // the automorphism as its own launch, from a temporary
      tmp = alloc(nc, level + 1, B);
      dst = lsq(tmp, 0, nc, level);
    }
    auto epilogue = [&](NttIO& io) {
      io.epi = !scatter ? NTT_EPI_SUBSCALE : aut_acc ? NTT_EPI_SUBSCALE_AUT_ACC : NTT_EPI_SUBSCALE_AUT;
      if (scatter) {  // a scatter in place would overwrite ex words other rows still read
        if (dst.p == x.p) throw std::runtime_error("moddown: the automorphism epilogue cannot run in place");
        io.aut = aut_index(galois_inverse(aut_g));
      }
      io.ex = limbs(x, 0, level + 1);
      const std::vector<u64> pq = p_mod_q(level);
      for (int j = 0; j <= level; ++j) {
        io.s[j] = hm_invmod(pq[j], mods[j]);
        io.ss[j] = hm_shoup(io.s[j], mods[j]);
      }
    };
    if (fused) {
      // the extension of the P limbs formed in the prologue of the NTT whose
      // epilogue is (x_Q - .) * P^-1: no basis_ext launch, no extended limbs in HBM
      NttIO io = nio(dst, xp);
      io.pro = NTT_PRO_BEXT;
      io.bx = moddown_tab(level);
      for (int j = 0; j <= level; ++j) io.bx_tab[j] = 0, io.bx_t[j] = (unsigned char)j;
      io.bx_s0[0] = 0;
      epilogue(io);
      intt_then_fwd(nio(xp, xp), io, K, K, rows_done);
    } else {
      if (rows_done) throw std::runtime_error("moddown: rows pass done, but the fused path is not taken");
      ntt(xp, true);
      Poly ext = alloc(nc, level + 1, B);
      LimbSet le = lsq(ext, 0, nc, level);
      {
        Scope sc(this, P_BEXT, 8.0 * N * B * nc * (K + level + 1));
        if (orion_launch_basis_ext(le, xp, moddown_tab(level), d_tb, N, stream))
          throw std::runtime_error("basis_ext: unsupported source count");
      }
      NttIO io = nio(dst, le);  // NTT of the extension and (x_Q - .) * P^-1, fused
      epilogue(io);
      ntt_io(io, false);
    }
    if (aut_g && !scatter) automorph(out, dst, aut_g, aut_acc);
  }
  // full key switch of c (Q, level) -> (k0, k1) written to out comps 0/1 (Q, level);
  // add0/add1 (optional, Q limbs 0..level with out's batch geometry): added to
  // comps 0/1 of the result, folded into the gadget product as P * add; aut_g:
  // the result permuted by that Galois element's automorphism (moddown), and
  // added to out's comps 0/1 for aut_acc
  void keyswitch(const LimbSet& c, int level, int B, const Poly& key, int klvl, const Poly& out,
                 const u64* add0 = nullptr, const u64* add1 = nullptr, u64 aut_g = 0, bool aut_acc = false) {
    if (klvl < level) throw std::runtime_error("evaluation key made for a lower level");
    Poly u = alloc(2, level + 1 + K, B);
    // when the gadget product runs the ModDown INTT's rows pass, it can run
    // the decomposition NTT's forward rows pass too (ORION_MAC_FWD_ROWS)
    const bool rows_q = mac_fwd_rows && moddown_rows_fusable(lsqp(u, 0, 2, level, level), level,
                                                             lsq(out, 0, 2, level), aut_g, aut_acc);
    bool fwd_rows = false;
    Poly D = decompose(c, level, B, rows_q, &fwd_rows);
    const int beta = (level + 1 + K - 1) / K;
    const LimbSet uq = lsqp(u, 0, 2, level, level), oq = lsq(out, 0, 2, level);
    const bool rows = moddown_rows_fusable(uq, level, oq, aut_g, aut_acc);
    mac_groups(uq, 0, lsqp(D, 0, beta, level, level), 0, c, 0, {key.ptr()}, {klvl}, beta, add0, 0,
               add0 ? level + 1 : 0, add1, rows ? level + 1 : 0, fwd_rows);
    moddown(uq, level, oq, aut_g, aut_acc, rows);
  }
  std::vector<u64> p_mod_q(int level) const {
    std::vector<u64> v;
    for (int j = 0; j <= level; ++j) {
      u64 P = 1;
      for (int k = 0; k < K; ++k) P = hm_mulmod(P, mods[L + k] % mods[j], mods[j]);
      v.push_back(P);
    }
    return v;
  }

  // ---------------------------------------------------------------------------
  // ciphertext operators
  // ---------------------------------------------------------------------------
  Ciphertext new_ct(int level, int B, long double scale) {
    Ciphertext c;
    c.poly = alloc(2, level + 1, B);
    c.level = level;
    c.scale = scale;
    return c;
  }
  Ciphertext clone(const Ciphertext& a) {
    Ciphertext c = new_ct(a.level, a.poly.B, a.scale);
    copy(lsq(c.poly, 0, 2, a.level), lsq(a.poly, 0, 2, a.level));
    return c;
  }

  void rescale_inplace(Ciphertext& ct) {
    const int l = ct.level;
    if (l < 1) throw std::runtime_error("cannot rescale a level-0 ciphertext");
    const int B = ct.poly.B;
    LimbSet last = ls(ct.poly, 0, 2, {l}, {l});
    // (DivRoundByLastModulusNTT) prep of every other limb, NTT and (c - .) * q_l^-1, fused
    LimbSet cq = lsq(ct.poly, 0, 2, l - 1);
    NttIO io = nio(cq, last);
    io.pro = NTT_PRO_RESCALE;
    io.modL = l;
    io.epi = NTT_EPI_SUBSCALE;
    io.ex = cq;
    for (int j = 0; j < l; ++j) {
      io.s[j] = hm_invmod(mods[l] % mods[j], mods[j]);
      io.ss[j] = hm_shoup(io.s[j], mods[j]);
    }
    (void)B;
    intt_then_fwd(nio(last, last), io, 1);  // INTT of the last limb, then the prep + NTT + tail
    ct.level = l - 1;
    ct.scale /= (long double)mods[l];
  }

  int batch_of(int a, int b) const {
    if (a == b || b == 1) return a;
    if (a == 1) return b;
    throw std::runtime_error("batch size mismatch");
  }

  Ciphertext mul_relin(const Ciphertext& a, const Ciphertext& b) {
    if (!have_rlk) throw std::runtime_error("relinearization key not generated");
    const int level = std::min(a.level, b.level);
    const int B = batch_of(a.poly.B, b.poly.B);
    Poly d = alloc(3, level + 1, B);
    {
      LimbSet ld = lsq(d, 0, 3, level);
      // distinct bytes: both operands' 2 components and the 3 outputs; a
      // square (Quad's x * x, activation.py:55) reads one ciphertext
      const bool square = a.poly.ptr() == b.poly.ptr();
      Scope sc(this, P_TENSOR, 8.0 * N * (level + 1) * B * (square ? 5 : 7));
      orion_launch_tensor(ld, lsq(a.poly, 0, 2, level, B), lsq(b.poly, 0, 2, level, B), d_tb, N, stream);
    }
    Ciphertext out = new_ct(level, B, a.scale * b.scale);
    // (d0, d1) + keyswitch(d2): the addition is folded into the gadget product
    keyswitch(lsq(d, 2, 1, level), level, B, rlk, L - 1, out.poly, d.ptr(), d.ptr() + d.comp_stride());
    return out;
  }

  Ciphertext rotate(const Ciphertext& a, int k) { return apply_galois(a, galois_element(k)); }
  // sigma_{5^k}(a) into out's buffer (allocated here when it has none)
  void rotate_into(const Ciphertext& a, int k, Ciphertext& out) {
    const u64 g = galois_element(k);
    const int level = a.level, B = a.poly.B;
    const EvKey& key = galois_key(g, level);
    if (!out.poly.buf) out.poly = new_ct(level, B, a.scale).poly;
    out.level = level;
    keyswitch(lsq(a.poly, 1, 1, level), level, B, key.k, key.level, out.poly, a.poly.ptr(), nullptr, g);
  }
  // sigma_g(a): key switch of c1 with the Galois key of g, + c0, NTT-domain permutation
  // (g = 2N - 1 is the complex conjugation of the slots)
  Ciphertext apply_galois(const Ciphertext& a, u64 g) {
    const int level = a.level, B = a.poly.B;
    const EvKey& key = galois_key(g, level);
    // sigma_g((c0, 0) + keyswitch(c1)): the c0 addition folded into the gadget
    // product, the automorphism into the ModDown's store
    Ciphertext out = new_ct(level, B, a.scale);
    keyswitch(lsq(a.poly, 1, 1, level), level, B, key.k, key.level, out.poly, a.poly.ptr(), nullptr, g);
    return out;
  }

  // a += sigma_{5^k}(a), in place: RotateNew(a, k) followed by
  // AddCiphertext(a, that rotation), with the addition in the ModDown's store
  // (c1 is decomposed and c0 folded into the gadget product before the ModDown
  // writes a)
  void rotate_add_inplace(Ciphertext& a, int k) {
    const u64 g = galois_element(k);
    const int level = a.level, B = a.poly.B;
    const EvKey& key = galois_key(g, level);
    keyswitch(lsq(a.poly, 1, 1, level), level, B, key.k, key.level, a.poly, a.poly.ptr(), nullptr, g, true);
  }

  // scale matching for additions (Lattigo evaluateInPlace: the lower-scale
  // operand is multiplied by the rounded integer ratio when it is > 1)
  void add_like(Ciphertext& out, const Ciphertext& a, const LimbSet& b, long double bscale, int op) {
    const int level = out.level;
    LimbSet o = lsq(out.poly, 0, 2, level);
    LimbSet la = lsq(a.poly, 0, 2, level, out.poly.B);
    long double ratio = a.scale > bscale ? a.scale / bscale : bscale / a.scale;
    long long r = llroundl(ratio);
    if (r > 1) {
      std::vector<u64> sc;
      for (int j = 0; j <= level; ++j) sc.push_back((u64)r % mods[j]);
      if (a.scale > bscale) {
        Poly tb = alloc(b.ncomp, level + 1, out.poly.B);
        LimbSet lt = lsq(tb, 0, b.ncomp, level);
        ew1(EW_SCALE, lt, b, &sc);
        ew(op, lsq(out.poly, 0, b.ncomp, level), lsq(a.poly, 0, b.ncomp, level, out.poly.B), lt);
        if (b.ncomp == 1 && &out != &a) copy(lsq(out.poly, 1, 1, level), lsq(a.poly, 1, 1, level, out.poly.B));
        out.scale = a.scale;
        return;
      }
      ew1(EW_SCALE, o, la, &sc);
      ew(op, lsq(out.poly, 0, b.ncomp, level), lsq(out.poly, 0, b.ncomp, level), b);
      out.scale = bscale;
      return;
    }
    ew(op, lsq(out.poly, 0, b.ncomp, level), lsq(a.poly, 0, b.ncomp, level, out.poly.B), b);
    if (b.ncomp == 1 && &out != &a) copy(lsq(out.poly, 1, 1, level), lsq(a.poly, 1, 1, level, out.poly.B));
    out.scale = a.scale;
  }

  // device plan of a BSGS transform: register slot of each baby, giant order,
  // and the diagonal plane of every (giant, slot) term
  void build_plan(LinTrans& T) {
    no_capture("building a linear transform's BSGS plan");
    T.slots.clear();
    T.gorder.clear();
    bool b0 = false, g0 = false;
    for (int b : T.babies) (b == 0 ? b0 = true : (T.slots.push_back(b), false));
    if (b0) T.slots.push_back(0);
    for (int j : T.giants) (j == 0 ? g0 = true : (T.gorder.push_back(j), false));
    if (g0) T.gorder.push_back(0);
    if ((int)T.slots.size() > LT_MAXSLOT)
      throw std::runtime_error("linear transform with more than 64 baby steps");
    std::map<int, int> slot_of;
    for (size_t s = 0; s < T.slots.size(); ++s) slot_of[T.slots[s]] = (int)s;
    const int ng = (int)T.gorder.size();
    const int nplan = (ng + LT_MAXG - 1) / LT_MAXG;
    std::vector<LtPlan> plans(nplan);
    memset(plans.data(), 0, plans.size() * sizeof(LtPlan));
    // operand copies of the diagonals in lt_bsgs's split-MAC form (the
    // diagonals themselves stay canonical for serialisation)
    T.sdiags.clear();
    for (auto& kv : T.diags) {
      const Poly& src = kv.second.poly;
      Poly dst = alloc(src.ncomp, src.nlimb, src.B);
      std::vector<int> md;
      for (int j = 0; j < src.nlimb; ++j) md.push_back(qp_mod(T.level, j));
      ew(EW_SPLIT24, ls(dst, 0, 1, iota(0, src.nlimb), md), ls(src, 0, 1, iota(0, src.nlimb), md),
         ls(src, 0, 1, iota(0, src.nlimb), md));
      T.sdiags.emplace(kv.first, dst);
    }
    // a zero diagonal in every plan slot a giant does not use, so lt_bsgs can
    // run its slots without per-slot branches (LT_DENSE; the products with it
    // add zero)
    {
      if (T.sdiags.empty()) throw std::runtime_error("linear transform has no diagonals loaded");
      const Poly& any = T.sdiags.begin()->second;
      Poly z = alloc(any.ncomp, any.nlimb, any.B);
      HIPCHK(hipMemsetAsync(z.ptr(), 0, (size_t)any.ncomp * any.nlimb * any.B * N * sizeof(u64), stream));
      T.sdiags.emplace(-1, z);
    }
    for (auto& P : plans)
      for (int gg = 0; gg < LT_MAXG; ++gg)
        for (int sl = 0; sl < LT_MAXSLOT; ++sl) P.pt[gg][sl] = T.sdiags.at(-1).ptr();
    for (int gi = 0; gi < ng; ++gi) {
      LtPlan& P = plans[gi / LT_MAXG];
      const int j = T.gorder[gi], gg = gi % LT_MAXG;
      for (int b : T.index.at(j)) {
        const int sl = slot_of.at(b);
        P.mask[gg] |= 1ull << sl;
        P.pt[gg][sl] = T.sdiags.at((j + b) & (slots - 1)).ptr();
      }
    }
    // a plan that a captured graph still holds is never rewritten: the graph
    // keeps replaying the plan (and the diagonals) it was captured with
    if (!T.plan || T.n_plan != nplan || T.plan.use_count() > 1) {
      void* d = nullptr;
      HIPCHK(hipMalloc(&d, nplan * sizeof(LtPlan)));
      T.plan = std::shared_ptr<void>(d, [](void* q) { hipFree(q); });
      T.d_plan = (LtPlan*)d;
    }
    h2d(T.d_plan, plans.data(), nplan * sizeof(LtPlan));
    T.n_plan = nplan;
    T.plan_dirty = false;
  }
  // the device plans of every transform whose diagonals are all loaded (a
  // pipeline reads the scheme's transforms and never builds their plans)
  void build_dirty_plans() {
    for (int id : lts.live()) {
      LinTrans& T = lts.get(id);
      if (!T.plan_dirty || T.giants.empty()) continue;
      bool all = true;
      for (int d : T.idx) all = all && T.diags.count(d & (slots - 1));
      if (all) build_plan(T);
    }
  }

  // BSGS linear transform (lintrans MultiplyByDiagMatrixBSGS restated; oracle_lt_bsgs).
  // Every phase runs as one grouped launch over all babies / all giants:
  //   1. one hoisted decomposition of ct1;
  //   2. all baby key switches (one MAC, decomposition shared) and their
  //      automorphisms with the + P*ct0 term (one launch);
  //   3. all giant inner products sum_s pt * rot_s (lt_bsgs: each baby read once);
  //   4. all giant key switches: ModDown of c1, decomposition, MAC with each
  //      giant's key (+ c0 folded in), then the automorphism-accumulate;
  //   5. ModDown of the accumulator.
  Ciphertext eval_lt(LinTrans& T, const Ciphertext& ct) {
    const int level = std::min(ct.level, T.level);
    const int B = ct.poly.B, nqp = level + 1 + K;
    const int beta = (level + 1 + K - 1) / K;
    if (T.giants.empty()) throw std::runtime_error("linear transform without diagonals");
    for (int d : T.idx)
      if (!T.diags.count(d & (slots - 1)))
        throw std::runtime_error("linear transform diagonal " + std::to_string(d) +
                                 " is not loaded (io_mode load: call LoadPlaintextDiagonal first)");
    if (T.plan_dirty) build_plan(T);
    const std::vector<u64> pq = p_mod_q(level);
    const int nb = (int)T.slots.size();
    const int nzb = nb - (T.slots.back() == 0 ? 1 : 0);

    // 1. hoisted decomposition of ct1 (only needed when some baby rotates)
    Poly D = nzb > 0 ? decompose(lsq(ct.poly, 1, 1, level), level, B) : alloc(1, 1, 1);
    LimbSet dl = lsqp(D, 0, 1, level, level);
    if (nzb == 0) dl.p = nullptr;
    LimbSet ctl = lsq(ct.poly, 0, 2, level);

    // 2-3. baby rotations + giant inner products (lt_bsgs): Tt comps [0, ng) =
    // c0 of giant slot gi, [ng, 2ng) = its c1
    const int ng = (int)T.gorder.size();
    const bool has_g0 = T.gorder.back() == 0;
    const int nzg = ng - (has_g0 ? 1 : 0);
    Poly Tt = alloc(2 * ng, nqp, B);
    {
      const Poly& pt0 = T.diags.begin()->second.poly;
      LimbSet ptl = lsqp(pt0, 0, 1, level, T.level, 1);
      for (int s0 = 0; s0 < nb; s0 += LT_MAXB) {
        LtBabies Bb;
        memset(&Bb, 0, sizeof(Bb));
        Bb.nb = std::min(LT_MAXB, nb - s0);
        Bb.s0 = s0;
        Bb.xcd = lt_xcd && (N / 256) % 8 == 0;
        Bb.beta = beta;
        Bb.K = K;
        Bb.level = level;
        Bb.L = L;
        for (int j = 0; j <= level; ++j) Bb.pq[j] = pq[j], Bb.pqs[j] = hm_shoup(pq[j], mods[j]);
        int nrot = 0;
        for (int s = 0; s < Bb.nb; ++s) {
          const int b = T.slots[s0 + s];
          if (b == 0) continue;
          const u64 g = galois_element(b);
          const EvKey& kk = galois_key(g, level);
          Bb.key[s] = kk.k.ptr();
          Bb.klvl[s] = kk.level;
          Bb.idx[s] = aut_index(g);
          ++nrot;
        }
        for (int p = 0; p < T.n_plan; ++p) {
          const int gcount = std::min(LT_MAXG, ng - p * LT_MAXG);
          LimbSet t0 = lsqp(Tt, p * LT_MAXG, 1, level, level), t1 = lsqp(Tt, ng + p * LT_MAXG, 1, level, level);
          // distinct bytes: the shared decomposition (beta digits) and ct0/ct1
          // once per row, the giant outputs (read back when accumulating), and
          // per QP limb the baby keys (2 beta each) and the diagonals of the
          // plan's (giant, baby) terms, both shared by the batch
          const double rows = (double)nqp * B;
          int npair = 0;
          for (int gi = p * LT_MAXG; gi < p * LT_MAXG + gcount; ++gi)
            for (int b : T.index.at(T.gorder[gi]))
              for (int s = 0; s < Bb.nb; ++s)
                if (T.slots[s0 + s] == b) ++npair;
          Scope sc(this, P_LTMAC,
                   8.0 * N * (rows * ((nzb ? beta : 0) + 2.0 + 2.0 * gcount * (s0 ? 2 : 1)) +
                              (double)nqp * (2.0 * beta * nrot + npair)));
          if (orion_launch_lt_bsgs(t0, t1, dl, ctl, Bb, T.d_plan + p, 0, gcount, s0 > 0, ptl, d_tb, N, stream))
            throw std::runtime_error("lt_bsgs launch failed");
        }
      }
    }

    // 4. giant key switches and the automorphism-accumulation (lt_giant)
    Poly acc = alloc(2, nqp, B);
    LimbSet la = lsqp(acc, 0, 2, level, level);
    Ciphertext out = new_ct(level, B, ct.scale * (long double)mods[T.level]);
    const LimbSet lo = lsq(out.poly, 0, 2, level);
    // one lt_giant launch: it may store the P limbs through the final
    // ModDown INTT's rows pass (as keyswitch's gadget product does)
    const bool rows = nzg > 0 && nzg <= ORION_MAXGROUP && moddown_rows_fusable(la, level, lo, 0, false);
    LimbSet z = lsqp(Tt, ng - 1, 2, level, level);  // the zero giant: (c0, c1) at comps ng-1, 2ng-1
    z.comp_stride = (long long)ng * Tt.comp_stride();
    if (nzg > 0) {
      Poly T1q = alloc(nzg, level + 1, B);
      moddown(lsqp(Tt, ng, nzg, level, level), level, lsq(T1q, 0, nzg, level));
      Poly Dg = decompose(lsq(T1q, 0, nzg, level), level, B);
      for (int g0 = 0; g0 < nzg; g0 += ORION_MAXGROUP) {
        LtGiants G;
        memset(&G, 0, sizeof(G));
        G.ng = std::min(ORION_MAXGROUP, nzg - g0);
        G.beta = beta;
        G.K = K;
        G.level = level;
        G.L = L;
        G.has_zero = (has_g0 && g0 == 0) ? 1 : 0;
        G.xcd = lt_xcd && (N / 256) % 8 == 0;
        G.rows_from = rows ? level + 1 : 0;
        G.logN = logN;
        G.d_gstride = (long long)beta * Dg.comp_stride();
        G.own_gstride = T1q.comp_stride();
        G.t0_gstride = Tt.comp_stride();
        for (int k = 0; k < G.ng; ++k) {
          const u64 g = galois_element(T.gorder[g0 + k]);
          const EvKey& kk = galois_key(g, level);
          G.key[k] = kk.k.ptr();
          G.klvl[k] = kk.level;
          G.idx[k] = aut_index(g);
        }
        LimbSet dg = lsqp(Dg, g0 * beta, 1, level, level);
        LimbSet own = lsq(T1q, g0, 1, level);
        LimbSet t0 = lsqp(Tt, g0, 1, level, level);
        LimbSet a = la;
        Poly part;
        if (g0 > 0) {  // > 64 giants: accumulate partial sums
          part = alloc(2, nqp, B);
          a = lsqp(part, 0, 2, level, level);
        }
        // per row: each giant's decomposition (beta) and t0 term, the output
        // pair and the zero giant; per QP limb: each giant's key (2 beta)
        const double rows = (double)nqp * B;
        Scope sc(this, P_LTGIANT, 8.0 * N * (rows * (G.ng * (beta + 1.0) + 2.0 + 2.0 * G.has_zero) +
                                          (double)nqp * 2.0 * beta * G.ng));
        if (orion_launch_lt_giant(a, dg, own, t0, z, G, d_tb, N, stream))
          throw std::runtime_error("lt_giant launch failed");
        if (g0 > 0) ew(EW_ADD, la, la, a);
      }
    } else {
      copy(la, z);
    }
    // 5.
    moddown(la, level, lo, 0, false, rows);
    return out;
  }

  // ---------------------------------------------------------------------------
  // encoder / encryptor
  // ---------------------------------------------------------------------------
  // values: B images x nvals float32 slots, device memory (encoder.hip);
  // limbs Q 0..level (+ P when qp)
  Plaintext encode_dev(const float* dvals, int nvals, int B, int level, long double scale, bool qp) {
    const int n = slots;
    if (nvals > n) throw std::runtime_error("too many values for the slot count");
    std::vector<int> md = iota(0, level + 1);
    if (qp)
      for (int k = 0; k < K; ++k) md.push_back(L + k);
    const int nl = (int)md.size();
    Plaintext pt;
    pt.level = level;
    pt.scale = scale;
    pt.qp = qp;
    pt.poly = alloc(1, nl, B);
    Buffer v(&pool, (size_t)B * n * sizeof(double2));
    const LimbSet out = ls(pt.poly, 0, 1, iota(0, nl), md);
    if (orion_launch_encode(dvals, nvals, B, (double2*)v.p, tw_inv, ci ? logN : logN - 1, ci, out, (double)scale,
                            d_tb, stream))
      throw std::runtime_error("encode launch failed");
    ntt(out, false);
    return pt;
  }
  Plaintext encode(const float* values, int nvals, int B, int level, long double scale, bool qp) {
    if (nvals > slots) throw std::runtime_error("too many values for the slot count");
    Buffer dv(&pool, (size_t)B * nvals * sizeof(float) + 16);
    HIPCHK(hipMemcpyAsync(dv.p, values, (size_t)B * nvals * sizeof(float), hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return encode_dev((const float*)dv.p, nvals, B, level, scale, qp);
  }

  // Garner table of `level`: inv[j][k] = (q_k mod q_j)^-1 mod q_j, then the
  // mixed-radix digits of floor((Q - 1) / 2)
  const u64* garner_table(int level) {
    auto it = garner.find(level);
    if (it != garner.end()) return it->second;
    no_capture("a decode CRT table");
    const int nl = level + 1;
    std::vector<u64> t((size_t)nl * nl + nl, 0);
    for (int j = 0; j < nl; ++j)
      for (int k = 0; k < j; ++k) t[(size_t)j * nl + k] = hm_invmod(mods[k] % mods[j], mods[j]);
    u64 rem = 0;
    for (int j = nl - 1; j >= 0; --j) {
      const u128 cur = (u128)rem * mods[j] + (mods[j] - 1);
      t[(size_t)nl * nl + j] = (u64)(cur / 2);
      rem = (u64)(cur % 2);
    }
    u64* d;
    HIPCHK(hipMalloc(&d, t.size() * sizeof(u64)));
    h2d(d, t.data(), t.size() * sizeof(u64));
    garner[level] = d;
    return d;
  }
  // slots (real parts) of every image into device memory out[B][slots]
  void decode_dev(const Plaintext& pt, double* out) {
    const int level = pt.level, B = pt.poly.B, nl = level + 1;
    if (nl > ORION_MAXLIMB) throw std::runtime_error("decode: too many limbs");
    Poly t = alloc(1, nl, B);
    const LimbSet x = lsq(t, 0, 1, level);
    ntt_io(nio(x, lsq(pt.poly, 0, 1, level)), true);
    Buffer v(&pool, (size_t)B * slots * sizeof(double2));
    if (orion_launch_decode(x, garner_table(level), (double)pt.scale, ci ? logN : logN - 1, ci, (double2*)v.p, tw_fwd,
                            out, d_tb, stream))
      throw std::runtime_error("decode launch failed");
  }
  std::vector<double> decode(const Plaintext& pt) {
    const size_t cnt = (size_t)pt.poly.B * slots;
    Buffer d(&pool, cnt * sizeof(double));
    decode_dev(pt, (double*)d.p);
    std::vector<double> out(cnt);
    HIPCHK(hipMemcpyAsync(out.data(), d.p, cnt * sizeof(double), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return out;
  }

  // public-key encryption (Lattigo rlwe Encryptor.EncryptZero + pt):
  // c0 = u pk0 + e0 + m, c1 = u pk1 + e1; u, e0, e1 sampled on the GPU
  Ciphertext encrypt(const Plaintext& pt) {
    if (!have_pk) throw std::runtime_error("public key not generated");
    const int level = pt.level, B = pt.poly.B;
    Poly r = alloc(3, level + 1, B);
    const LimbSet rs = lsq(r, 0, 3, level);
    if (orion_launch_enc_sample(rs, enc_sampler, d_tb, N, stream)) throw std::runtime_error("sampler launch failed");
    enc_sampler.enc += 1;
    ntt(rs, false);
    Ciphertext ct = new_ct(level, B, pt.scale);
    LimbSet c0 = lsq(ct.poly, 0, 1, level), c1 = lsq(ct.poly, 1, 1, level);
    ew(EW_MUL, c0, lsq(r, 0, 1, level), lsq(pk, 0, 1, level, B));
    ew(EW_ADD, c0, c0, lsq(r, 1, 1, level));
    ew(EW_ADD, c0, c0, lsq(pt.poly, 0, 1, level, B));
    ew(EW_MUL, c1, lsq(r, 0, 1, level), lsq(pk, 1, 1, level, B));
    ew(EW_ADD, c1, c1, lsq(r, 2, 1, level));
    return ct;
  }

  Plaintext decrypt(const Ciphertext& ct) {
    if (!have_sk) throw std::runtime_error("secret key not generated");
    const int level = ct.level, B = ct.poly.B;
    Plaintext pt;
    pt.level = level;
    pt.scale = ct.scale;
    pt.poly = alloc(1, level + 1, B);
    LimbSet p = lsq(pt.poly, 0, 1, level);
    ew(EW_MUL, p, lsq(ct.poly, 1, 1, level), lsq(sk, 0, 1, level, B));
    ew(EW_ADD, p, p, lsq(ct.poly, 0, 1, level));
    return pt;
  }

  // rounded integer constant c -> residues at `level`
  std::vector<u64> const_residues(long double c, int level) const {
    std::vector<u64> r;
    const bool neg = c < 0;
    long double a = neg ? -c : c;
    // a < 2^64 required
    if (a >= 18446744073709551615.0L) throw std::runtime_error("scalar constant too large");
    const u64 v = (u64)a;
    for (int j = 0; j <= level; ++j) {
      const u64 x = v % mods[j];
      r.push_back(neg ? (x ? mods[j] - x : 0) : x);
    }
    return r;
  }
  // round(c) (half away from zero) of any magnitude -> residues at `level`;
  // |c| >= 2^63 is an integer m 2^e (64-bit long double mantissa), reduced exactly
  std::vector<u64> big_const_residues(long double c, int level) const {
    const bool neg = c < 0;
    long double a = floorl((neg ? -c : c) + 0.5L);
    u64 m;
    int e = 0;
    if (a >= 9223372036854775808.0L) {
      int ex;
      const long double fr = frexpl(a, &ex);
      m = (u64)ldexpl(fr, 64);
      e = ex - 64;
    } else {
      m = (u64)a;
    }
    std::vector<u64> r;
    for (int j = 0; j <= level; ++j) {
      const u64 q = mods[j];
      const u64 x = hm_mulmod(m % q, hm_powmod(2 % q, (u64)e, q), q);
      r.push_back(neg ? (x ? q - x : 0) : x);
    }
    return r;
  }

  // ---------------------------------------------------------------------------
  // polynomial evaluation (polyeval.go:63-84 -> Lattigo v6 he.EvaluatePolynomial,
  // restated): p(x) in the monomial or Chebyshev basis, consuming exactly
  // bitlen(degree) levels (orion/nn/activation.py:22-23,106-107 plans for that)
  // and returning exactly the requested scale.
  //   * power basis (PowerBasis.GenPower): T_{2s} = T_s^2 (Chebyshev
  //     2 T_s^2 - 1); baby steps T_j from a = 2^k - 1, b = j + 1 - 2^k
  //     (Chebyshev 2 T_a T_b - T_|a-b|, T_c scaled by round(s_a s_b / s_c)
  //     before the rescale); every stored power is rescaled once.  Babies are
  //     made on first use (Lattigo makes all j < 2^logSplit up front; the
  //     values are the same);
  //   * Paterson-Stockmeyer tree (GetPatersonStockmeyerPolynomial /
  //     recursePS): logSplit = OptimalSplit(bitlen(deg)), top target level
  //     level(x) - bitlen(deg) + 1.  A node of degree < 2^logSplit is a leaf,
  //     except that a lead node (the chain of quotients from the top) whose
  //     MaxDeg > 2^bitlen(MaxDeg) - 2^(logSplit-1) is re-split with
  //     logSplit = OptimalSplit(bitlen(deg)), passed down to its subtree.
  //     Otherwise p = q X^m + r, m = the smallest power of two >= 2^logSplit
  //     and >= deg/2 + 1 (Chebyshev: T_{m+j} = 2 T_m T_j - T_{m-j});
  //   * scales (ckks simEvaluator.UpdateLevelAndScale{Baby,Giant}Step): the q
  //     branch runs one level up at scale S q_i / scale(X^m), q_i = q_level
  //     for a lead node and q_{level+1} otherwise; its result is rescaled and
  //     multiplied by X^m, and the r branch runs at that product's scale; a
  //     lead leaf is evaluated at S q_level.  The top result is rescaled once,
  //     landing on the target scale;
  //   * a leaf (EvaluatePolynomialVectorFromPowerBasis) is c_0 S + sum_j
  //     round(c_j S / scale(T_j)) T_j (MulThenAdd: half away from zero), at
  //     the lowest level among its target and the powers it uses, as
  //     MulThenAdd and Add take the lower level of their operands.
  // ---------------------------------------------------------------------------
  struct PolyFn {
    bool cheb = false;
    std::vector<long double> c;  // lowest degree first
  };
  struct PolyRun {
    const Ciphertext* x;
    bool cheb;
    std::map<int, Ciphertext> pw;    // T_{2^k}, k >= 1
    std::map<int, Ciphertext> baby;  // T_j, j not a power of two
  };
  static int ceil_log2(int j) {
    int k = 0;
    while ((1 << k) < j) ++k;
    return k;
  }
  static int optimal_split(int logd) {  // Lattigo bignum.OptimalSplit
    int ls = logd >> 1;
    const int a = (1 << ls) + (1 << (logd - ls)) + logd - ls - 3;
    const int b = (1 << (ls + 1)) + (1 << (logd - ls - 1)) + logd - ls - 4;
    if (a > b) ++ls;
    return ls;
  }
  const Ciphertext& poly_T(PolyRun& R, int j) {
    if (j == 1) return *R.x;
    if ((j & (j - 1)) == 0) return R.pw.at(j);
    auto it = R.baby.find(j);
    if (it != R.baby.end()) return it->second;
    const int k = ceil_log2(j) - 1, a = (1 << k) - 1, b = j + 1 - (1 << k), c = a > b ? a - b : b - a;
    const Ciphertext& A = poly_T(R, a);
    const Ciphertext& Bc = poly_T(R, b);
    Ciphertext t = mul_relin(A, Bc);
    if (R.cheb) {
      const LimbSet lt = lsq(t.poly, 0, 2, t.level);
      ew(EW_ADD, lt, lt, lt);
      if (c == 0) {
        std::vector<u64> one = big_const_residues(-t.scale, t.level);
        ew1(EW_ADDC, lsq(t.poly, 0, 1, t.level), lsq(t.poly, 0, 1, t.level), &one);
      } else {
        const Ciphertext& C = poly_T(R, c);
        std::vector<u64> k = big_const_residues(-(t.scale / C.scale), t.level);
        ew(EW_ADDSCALE, lt, lsq(C.poly, 0, 2, t.level), lt, &k);
      }
    }
    rescale_inplace(t);
    return R.baby.emplace(j, std::move(t)).first->second;
  }
  static std::pair<std::vector<long double>, std::vector<long double>> poly_split(const std::vector<long double>& c,
                                                                                  int s, bool cheb) {
    const int deg = (int)c.size() - 1;
    std::vector<long double> q(c.begin() + s, c.end()), r(c.begin(), c.begin() + s);
    if (cheb) {
      for (int j = 1; j <= deg - s; ++j) {
        q[j] = 2 * c[s + j];
        r[s - j] -= c[s + j];
      }
    }
    return {q, r};
  }
  // leaf: c_0 S + sum_j round(c_j S / scale(T_j)) T_j at level min(lam, level(T_j))
  Ciphertext poly_leaf(PolyRun& R, const std::vector<long double>& c, int lam, long double S) {
    const int deg = (int)c.size() - 1, B = R.x->poly.B;
    int lv = lam;
    for (int j = 1; j <= deg; ++j)
      if (c[j] != 0) lv = std::min(lv, poly_T(R, j).level);
    Ciphertext o = new_ct(lv, B, S);
    const LimbSet lo = lsq(o.poly, 0, 2, lv);
    bool first = true;
    for (int j = 1; j <= deg; ++j) {
      if (c[j] == 0) continue;
      const Ciphertext& T = poly_T(R, j);
      std::vector<u64> k = big_const_residues(c[j] * S / T.scale, lv);
      ew1(first ? EW_SCALE : EW_ADDSCALE, lo, lsq(T.poly, 0, 2, lv), &k);
      first = false;
    }
    if (first) HIPCHK(hipMemsetAsync(o.poly.ptr(), 0, (size_t)2 * (lv + 1) * B * N * sizeof(u64), stream));
    if (c[0] != 0) {
      std::vector<u64> k = big_const_residues(c[0] * S, lv);
      ew1(EW_ADDC, lsq(o.poly, 0, 1, lv), lsq(o.poly, 0, 1, lv), &k);
    }
    return o;
  }
  static int bitlen(int v) {
    int k = 0;
    while (v >> k) ++k;
    return k;
  }
  // recursePS: node c (lead: on the quotient chain from the top; maxdeg as
  // splitCoeffs propagates it) evaluated for target level lam and scale S
  Ciphertext poly_ps(PolyRun& R, const std::vector<long double>& c, bool lead, int maxdeg, int logSplit, int lam,
                     long double S) {
    const int deg = (int)c.size() - 1;
    if (deg < (1 << logSplit)) {
      if (lead && logSplit > 1 && maxdeg > (1 << bitlen(maxdeg)) - (1 << (logSplit - 1)))
        return poly_ps(R, c, lead, maxdeg, optimal_split(bitlen(deg)), lam, S);
      return poly_leaf(R, c, lam, lead ? S * (long double)mods[lam] : S);
    }
    int m = 1 << logSplit;
    while (m < (deg >> 1) + 1) m <<= 1;
    auto qr = poly_split(c, m, R.cheb);
    const int rmax = maxdeg == deg ? m - 1 : maxdeg - (deg - m + 1);
    const Ciphertext& X = R.pw.at(m);
    if (lam + 1 > R.x->level) throw std::runtime_error("polynomial evaluation: level plan violated");
    const long double qi = (long double)mods[lead ? lam : lam + 1];
    Ciphertext qc = poly_ps(R, qr.first, lead, maxdeg, logSplit, lam + 1, S * qi / X.scale);
    rescale_inplace(qc);
    Ciphertext o = mul_relin(qc, X);
    Ciphertext rc = poly_ps(R, qr.second, false, rmax, logSplit, lam, o.scale);
    const int lv = std::min(o.level, rc.level);  // Add takes the lower level
    o.level = lv;
    const LimbSet lo = lsq(o.poly, 0, 2, lv);
    ew(EW_ADD, lo, lo, lsq(rc.poly, 0, 2, lv));
    return o;
  }
  Ciphertext eval_poly(const Ciphertext& x, const PolyFn& p, long double target) {
    const int deg = (int)p.c.size() - 1;
    if (deg < 0) throw std::runtime_error("empty polynomial");
    const int depth = bitlen(deg);  // bits.Len64(degree)
    if (x.level < depth)
      throw std::runtime_error(std::to_string(x.level) + " levels < " + std::to_string(depth) +
                               " log(d) -> cannot evaluate poly");
    PolyRun R;
    R.x = &x;
    R.cheb = p.cheb;
    for (int s = 1; 2 * s <= deg; s *= 2) {
      const Ciphertext& a = s == 1 ? x : R.pw.at(s);
      Ciphertext t = mul_relin(a, a);
      rescale_inplace(t);
      if (p.cheb) {
        const LimbSet lt = lsq(t.poly, 0, 2, t.level);
        ew(EW_ADD, lt, lt, lt);
        std::vector<u64> one = big_const_residues(-t.scale, t.level);
        ew1(EW_ADDC, lsq(t.poly, 0, 1, t.level), lsq(t.poly, 0, 1, t.level), &one);
      }
      R.pw.emplace(2 * s, std::move(t));
    }
    if (deg == 0) return poly_leaf(R, p.c, x.level, target);
    Ciphertext out = poly_ps(R, p.c, true, deg, optimal_split(depth), x.level - depth + 1, target);
    rescale_inplace(out);
    out.scale = target;
    return out;
  }
  HandlePool<PolyFn> polys;

  // ---------------------------------------------------------------------------
  // bootstrapping (bootstrapper.go:15-87).  As in Lattigo, a
  // bootstrapper is made per slot count (NewBootstrapper(logPs, slots)), and
  // its circuit runs under bootstrapping parameters of its own.  Orion sets
  // only LogN, LogP, Xs and LogSlots (bootstrapper.go:33-38); every other
  // field is Lattigo v6's default bootstrapping.ParametersLiteral [U]
  // (DESIGN.md §6 lists each default beside what is done here):
  //   CoeffsToSlots 4 levels of 56-bit primes, SlotsToCoeffs 3 levels of
  //   39-bit primes, EvalMod 60-bit primes, K = 16, Mod1 degree 30, 3 double
  //   angles, no arcsine (Mod1InvDegree 0), LogMessageRatio 8, an ephemeral
  //   secret of Hamming weight 32.
  // The chain is the residual Q chain + 3 x 39 + (bitlen(30) + 3) x 60 + 4 x
  // 56 bits, with key-switching P primes of the bit sizes logPs.  Those
  // parameters live in a second Context -- the bootstrapping context, one per
  // distinct logPs, shared by the slot counts -- that holds the same secret
  // and its own relinearisation and Galois keys; the scheme's context, chain
  // and keys are not touched.  The circuit, for n slots (gap = N / 2n), with
  // every constant derived from the parameters (oracle_bootstrap derives
  // them again, independently):
  //   ScaleDown: the level-0 residues times F = round(q0 / (2^8 Delta)), so
  //      the message sits 2^LogMessageRatio below q0
  //   -> EvkDenseToSparse at level 0 (key switch s -> s_eph, h(s_eph) = 32)
  //   -> ModRaise (level 0 -> top of the bootstrapping chain, t = m + q0 I
  //      with |I| small because s_eph is sparse)
  //   -> EvkSparseToDense at the top level (s_eph -> s)
  //   -> Trace, n < N/2 only: multiply by gap^-1 mod Q, then add the
  //      log2(gap) rotations by n 2^i (SubSum): the exact projection on
  //      Z[X^gap], whose slots are the n-periodic average of the input's
  //   -> CoeffsToSlots: the n-point special inverse FFT's butterfly stages
  //      merged into 4 BSGS transforms with complex diagonals (n-periodic; the
  //      extra stages go to the first transforms); the final bit reversal is
  //      skipped because EvalMod is slot-wise and SlotsToCoeffs starts with
  //      the matching one.  The 1/n and EvalMod's 1/(2K) are spread over the
  //      transforms.  For n < N/2 the last transform also packs: real parts
  //      into slots [0, n) and imaginary parts into [n, 2n) of every
  //      2n-period, so that one EvalMod serves both
  //   -> EvalMod: the degree-30 Chebyshev interpolant of
  //      a cos(2 pi (K u - 1/4) / 2^r) on [-1, 1], a = (2 pi)^(-1/2^r), at a
  //      target scale chosen so that after the r double angles
  //      y <- 2 y^2 - a^(2^(i+1)) (constant added before the rescale, as
  //      Lattigo's mod1 evaluator does) the scale is 2^60; the result is
  //      sin(2 pi x) / (2 pi) = F m / q0 + O(m^3); once (n < N/2) or on the
  //      real and the imaginary part (n = N/2, recombined with x i = X^(N/2))
  //   -> SlotsToCoeffs: the forward stages, 3 transforms carrying
  //      q0 / (F s_y) (for n < N/2 the first one also unpacks real + i imag)
  //      -> the residual top level, copied back into the scheme's context at
  //      the input's scale.
  // Bootstrap then applies Orion's post-scale 2^(LogMaxSlots - LogSlots)
  // (bootstrapper.go:73-74): an input whose slots >= n are zero comes back with
  // its n slots replicated over all N/2 (Lattigo's sparse packing).
  // ---------------------------------------------------------------------------
  typedef std::complex<double> cplx;
  typedef std::map<int, std::vector<cplx>> DiagMap;  // rotation offset -> diagonal (n slots)

  Plaintext encode_complex(const std::vector<cplx>& v, int level, long double scale, bool qp) {
    const int n = N / 2;
    std::vector<int> md = iota(0, level + 1);
    if (qp)
      for (int k = 0; k < K; ++k) md.push_back(L + k);
    const int nl = (int)md.size();
    Plaintext pt;
    pt.level = level;
    pt.scale = scale;
    pt.qp = qp;
    pt.poly = alloc(1, nl, 1);
    std::vector<double2> host(n);
    for (int i = 0; i < n; ++i) host[i] = make_double2(v[i].real(), v[i].imag());
    Buffer dv(&pool, (size_t)n * sizeof(double2));
    HIPCHK(hipMemcpyAsync(dv.p, host.data(), host.size() * sizeof(double2), hipMemcpyHostToDevice, stream));
    const LimbSet out = ls(pt.poly, 0, 1, iota(0, nl), md);
    if (orion_launch_encode_c((double2*)dv.p, 1, tw_inv, logN - 1, false, out, (double)scale, d_tb, stream))
      throw std::runtime_error("encode launch failed");
    HIPCHK(hipStreamSynchronize(stream));
    ntt(out, false);
    return pt;
  }
  // BSGS transform y = sum_d diag_d * rot(x, d) with complex diagonals encoded
  // at scale q_level; the bootstrapping DFT matrices' LogBSGSRatio is 1 [U]
  LinTrans make_lt_complex(const DiagMap& dm, int level) {
    const int slots = N / 2;
    LinTrans T;
    T.level = level;
    T.ratio = 2;
    for (auto& kv : dm) T.idx.push_back(kv.first);
    T.N1 = find_best_n1(T.idx, slots, 1);
    std::set<int> seenb;
    for (int d : T.idx) {
      int gi, bi;
      bsgs_split(d, slots, T.N1, &gi, &bi);
      T.index[gi].push_back(bi);
      if (!seenb.count(bi)) {
        seenb.insert(bi);
        T.babies.push_back(bi);
      }
    }
    for (auto& kv : T.index) {
      std::sort(kv.second.begin(), kv.second.end());
      T.giants.push_back(kv.first);
    }
    std::vector<cplx> vec(slots);
    for (auto& kv : dm) {
      int gi, bi;
      bsgs_split(kv.first, slots, T.N1, &gi, &bi);
      for (int s2 = 0; s2 < slots; ++s2) vec[s2] = kv.second[((s2 - gi) % slots + slots) % slots];
      T.diags[kv.first & (slots - 1)] = encode_complex(vec, level, (long double)mods[level], true);
    }
    return T;
  }
  // one butterfly stage of the special FFT as a diagonal map (offsets mod n)
  DiagMap fft_stage(int len, bool inverse, const std::vector<Cplx>& tw) const {
    const int n = N / 2, h = len / 2;
    DiagMap m;
    auto at = [&](int off) -> std::vector<cplx>& {
      auto it = m.find(off);
      if (it == m.end()) it = m.emplace(off, std::vector<cplx>(n, cplx(0, 0))).first;
      return it->second;
    };
    std::vector<cplx>&d0 = at(0), &dp = at(h), &dm = at(n - h);
    for (int p = 0; p < n; ++p) {
      const int j = p & (len - 1);
      if (j < h) {
        const cplx w = inverse ? cplx(1, 0) : cplx(tw[h + j].re, tw[h + j].im);
        d0[p] += 1.0;
        dp[p] += w;  // x_{p+h}
      } else {
        const cplx w(tw[h + j - h].re, tw[h + j - h].im);
        if (inverse) {  // (x_{p-h} - x_p) w
          dm[p] += w;
          d0[p] -= w;
        } else {  // x_{p-h} - w x_p
          dm[p] += 1.0;
          d0[p] -= w;
        }
      }
    }
    return m;
  }
  // (A o B): apply B, then A
  DiagMap diag_compose(const DiagMap& A, const DiagMap& Bm) const {
    const int n = N / 2;
    DiagMap C;
    for (auto& a : A)
      for (auto& b : Bm) {
        const int off = (a.first + b.first) % n;
        auto it = C.find(off);
        if (it == C.end()) it = C.emplace(off, std::vector<cplx>(n, cplx(0, 0))).first;
        for (int p = 0; p < n; ++p) it->second[p] += a.second[p] * b.second[(p + a.first) % n];
      }
    return C;
  }
  struct Bootstrapper {
    // Lattigo v6 bootstrapping.ParametersLiteral defaults [U]:
    // CoeffsToSlots / SlotsToCoeffs factorisation depths and prime sizes,
    // EvalMod prime size, Mod1 degree, double angles, K, LogMessageRatio and
    // the ephemeral secret's Hamming weight
    static constexpr int kCtS = 4, kCtSBits = 56, kStC = 3, kStCBits = 39, kModBits = 60;
    static constexpr int kDegree = 30, kR = 3, kK = 16, kLogMsgRatio = 8, kEphH = 32;
    static constexpr int kDepthPoly = 5;  // bits.Len64(kDegree)
    static constexpr int kLogBSGSRatio = 1;  // dft.MatrixLiteral LogBSGSRatio
    static_assert(kCtS == 4 && kStC == 3, "the constant spreading below takes 4th and cube roots");
    Context* bc = nullptr;  // the bootstrapping context (owned by the scheme's btp_ctx)
    int slots = 0, gap = 1, K = kK, r = kR, degree = kDegree;
    PolyFn cosp;
    long double t0 = 0;              // EvalMod polynomial target scale
    std::vector<long double> dac;    // double-angle constants a^(2^(i+1)), i < r
    std::vector<LinTrans> cts, stc;  // in application order
    std::vector<u64> trace_gal;      // Galois elements of the trace (rotations by slots * 2^i)
    int top = 0;
    Poly mono_i;          // n = N/2: NTT of X^(N/2) (x i on every slot), all Q limbs
    long double s_y = 0;  // scale of the EvalMod output (2^60 up to rounding)
    u64 F = 1;            // ScaleDown: message times F = round(q0 / (2^8 Delta)) before ModRaise
    EvKey d2s, s2d;       // EvkDenseToSparse (level 0), EvkSparseToDense (full chain)
  };
  // declared in this order so that the circuits (whose buffers belong to a
  // bootstrapping context's pool) are destroyed before the contexts
  std::map<std::vector<int>, std::unique_ptr<Context>> btp_ctx;  // logPs -> bootstrapping context
  std::map<int, std::unique_ptr<Bootstrapper>> btps;             // slot count -> circuit

  // the butterfly stages of the n-point special FFT (lengths in application
  // order) split over ng transforms, the extra stages to the first ones
  static std::vector<std::vector<int>> fft_groups(int ns, bool inverse, int ng) {
    std::vector<int> lens;
    for (int len = inverse ? ns : 2; inverse ? len >= 2 : len <= ns; len = inverse ? len / 2 : len * 2)
      lens.push_back(len);
    std::vector<std::vector<int>> g(ng);
    const int tot = (int)lens.size();
    int at = 0;
    for (int k = 0; k < ng; ++k)
      for (int i = 0; i < tot / ng + (k < tot % ng ? 1 : 0); ++i) g[k].push_back(lens[at++]);
    return g;
  }

  // (on the bootstrapping context) the circuit for `ns` slots
  std::unique_ptr<Bootstrapper> make_circuit(int ns) {
    typedef Bootstrapper BT;
    const int n = N / 2;
    auto B = std::unique_ptr<Bootstrapper>(new Bootstrapper());
    B->bc = this;
    B->slots = ns;
    B->gap = n / ns;
    const long double PI = 3.14159265358979323846264338327950288L;
    // EvalMod: Lattigo's default Mod1Type CosDiscrete [U] -- a cos(2 pi (x -
    // 1/4) / 2^r), a = (2 pi)^(-1/2^r), interpolated at nodes on the integers
    // the ModRaise overflow takes (x = K u; hostmath.cpp cos_discrete_cheb,
    // nodes within 2^-LogMessageRatio of each integer); after the r double
    // angles y <- 2 y^2 - a^(2^(i+1)) it is sin(2 pi x) / (2 pi)
    const long double a = powl(2 * PI, -1.0L / (long double)(1 << B->r));
    B->cosp.cheb = true;
    B->cosp.c = cos_discrete_cheb(B->K, B->degree, B->r, ldexp(1.0, -BT::kLogMsgRatio));
    {
      long double v = a;
      for (int i = 0; i < B->r; ++i) B->dac.push_back(v = v * v);
    }
    B->top = L - 1;
    {  // ScaleDown (LogMessageRatio): round(q0 / (2^8 Delta)), Delta the default scale
      const long double f = roundl((long double)mods[0] / ldexpl(1.0L, BT::kLogMsgRatio + logScale));
      B->F = f < 1 ? 1 : (u64)f;
    }
    for (int s = ns; s < n; s *= 2) B->trace_gal.push_back(galois_element(s));
    int logns = 0;
    while ((1 << logns) < ns) ++logns;
    // the n-point special FFT (slots of Z[Y]/(Y^2n + 1), Y = X^gap); its
    // diagonals act n-periodically on the N/2 slots
    const std::vector<Cplx> twi = special_fft_twiddles(logns + 1, true), twf = special_fft_twiddles(logns + 1, false);
    const bool packed = ns < n;
    // CoeffsToSlots: slots of t / q0 -> bitrev((t_j + i t_{j+n}) / q0) / (2K).  The 1/n of the
    // inverse transform and EvalMod's 1 / (2K) are spread over the transforms (2^-s per
    // transform of s stages, the 4th root of 1 / (2K) each), so no diagonal is small against
    // the fixed-point grid of its encoding
    {
      const auto g = fft_groups(ns, true, BT::kCtS);
      int level = B->top;
      const double kf = sqrt(sqrt(1.0 / (2.0 * B->K)));
      for (int k = 0; k < BT::kCtS; ++k) {
        DiagMap M;
        M[0] = std::vector<cplx>(n, cplx(ldexp(kf, -(int)g[k].size()), 0));
        for (int len : g[k]) M = diag_compose(fft_stage(len, true, twi), M);
        if (packed && k == BT::kCtS - 1) {
          // w -> a w, a = 1 on [0, n) and -i on [n, 2n) of every 2n-period: then
          // a w + conj(a w) = 2 Re w on the first half, 2 Im w on the second
          DiagMap A;
          A[0] = std::vector<cplx>(n);
          for (int p = 0; p < n; ++p) A[0][p] = (p % (2 * ns)) < ns ? cplx(1, 0) : cplx(0, -1);
          M = diag_compose(A, M);
        }
        B->cts.push_back(make_lt_complex(M, level--));
      }
    }
    // EvalMod scales: the polynomial's target t0 is chosen so that the r
    // double angles (rescaled by the primes below its output level) end on
    // 2^60; s_y is the scale they actually reach (the same long double steps
    // as mul_relin and rescale_inplace)
    {
      const int lp = B->top - BT::kCtS - BT::kDepthPoly;  // level of the polynomial's output
      long double T = ldexpl(1.0L, BT::kModBits);
      for (int i = B->r - 1; i >= 0; --i) T = sqrtl(T * (long double)mods[lp - i]);
      B->t0 = T;
      long double sc = T;
      for (int i = 0; i < B->r; ++i) sc = sc * sc / (long double)mods[lp - i];
      B->s_y = sc;
      // SlotsToCoeffs: forward stages times c = q0 / (F s_y), so the output decodes at the
      // input scale
      const auto g = fft_groups(ns, false, BT::kStC);
      int level = lp - B->r;
      const double cf = cbrt((double)((long double)mods[0] / ((long double)B->F * sc)));
      for (int k = 0; k < BT::kStC; ++k) {
        DiagMap M;
        if (packed && k == 0) {
          // unpack: y_p + i y_{p+n} on the first half of a 2n-period, i y_p + y_{p-n}
          // (= y_{p+n}: y is 2n-periodic) on the second, so the result is n-periodic
          M[0] = std::vector<cplx>(n);
          M[ns] = std::vector<cplx>(n);
          for (int p = 0; p < n; ++p) {
            const bool lo = (p % (2 * ns)) < ns;
            M[0][p] = lo ? cplx(cf, 0) : cplx(0, cf);
            M[ns][p] = lo ? cplx(0, cf) : cplx(cf, 0);
          }
        } else {
          M[0] = std::vector<cplx>(n, cplx(cf, 0));
        }
        for (int len : g[k]) M = diag_compose(fft_stage(len, false, twf), M);
        B->stc.push_back(make_lt_complex(M, level--));
      }
    }
    if (!packed) {  // x i on every slot = multiplication by X^(N/2)
      B->mono_i = alloc(1, L, 1);
      std::vector<u64> host((size_t)L * N, 0);
      for (int l = 0; l < L; ++l) host[(size_t)l * N + N / 2] = 1;
      upload(B->mono_i, host);
      ntt(lsq(B->mono_i, 0, 1, L - 1), false);
    }
    {  // the ephemeral secret and its keys (genEncapsulationEvaluationKeysNew)
      const Poly se = secret_poly(sample_ternary_h(BT::kEphH));
      B->d2s = EvKey{gen_evk(sk, se, 0), 0};
      B->s2d = EvKey{gen_evk(se, sk, L - 1), L - 1};
    }
    return B;
  }

  Ciphertext mul_i(const Bootstrapper& bt, const Ciphertext& a) {
    Ciphertext o = new_ct(a.level, a.poly.B, a.scale);
    LimbSet mi = ls(bt.mono_i, 0, 1, iota(0, a.level + 1), iota(0, a.level + 1), a.poly.B);
    mi.ncomp = 2;
    mi.comp_stride = 0;  // one plaintext for both components
    ew(EW_MUL, lsq(o.poly, 0, 2, a.level), lsq(a.poly, 0, 2, a.level), mi);
    return o;
  }
  Ciphertext lt_rescale(LinTrans& T, const Ciphertext& x) {
    Ciphertext y = eval_lt(T, x);
    rescale_inplace(y);
    y.scale = x.scale;  // diagonals at scale q_level
    return y;
  }
  // mod1 evaluator: the cosine polynomial, then the double angles
  // y <- 2 y^2 - a^(2^(k+1)), the constant added at the product's scale
  // before its rescale
  Ciphertext eval_mod(const Bootstrapper& bt, const Ciphertext& u) {
    Ciphertext y = eval_poly(u, bt.cosp, bt.t0);
    for (int k = 0; k < bt.r; ++k) {
      Ciphertext t = mul_relin(y, y);
      const LimbSet lt = lsq(t.poly, 0, 2, t.level);
      ew(EW_ADD, lt, lt, lt);
      std::vector<u64> c = big_const_residues(-bt.dac[k] * t.scale, t.level);
      ew1(EW_ADDC, lsq(t.poly, 0, 1, t.level), lsq(t.poly, 0, 1, t.level), &c);
      rescale_inplace(t);
      y = std::move(t);
    }
    return y;
  }
  // (on the bootstrapping context) x: the level-0 residues (NTT domain) of a
  // batch of B ciphertexts, already scaled down by F
  Ciphertext run_circuit(Bootstrapper& bt, const Poly& x, int B) {
    // EvkDenseToSparse at level 0: (x0, 0) + KS(x1), now under the ephemeral secret
    Poly e = alloc(2, 1, B);
    keyswitch(lsq(x, 1, 1, 0), 0, B, bt.d2s.k, bt.d2s.level, e, x.ptr());
    // ModRaise: the centred level-0 residues (coefficient domain) lifted to every Q limb
    Poly c0 = alloc(2, 1, B);
    ntt_io(nio(lsq(c0, 0, 2, 0), lsq(e, 0, 2, 0)), true);
    Ciphertext m = new_ct(L - 1, B, (long double)mods[0]);
    const LimbSet ml = lsq(m.poly, 0, 2, L - 1);
    if (orion_launch_modraise(ml, lsq(c0, 0, 2, 0), d_tb, N, stream)) throw std::runtime_error("modraise failed");
    ntt(ml, false);
    // EvkSparseToDense at the top level: (m0, 0) + KS(m1), back under the secret
    Ciphertext t = new_ct(L - 1, B, m.scale);
    keyswitch(lsq(m.poly, 1, 1, L - 1), L - 1, B, bt.s2d.k, bt.s2d.level, t.poly, m.poly.ptr());
    const LimbSet tl = lsq(t.poly, 0, 2, L - 1);
    if (bt.gap > 1) {  // Trace: (gap^-1 t) summed over the rotations by slots * 2^i
      std::vector<u64> gi(L);
      for (int l = 0; l < L; ++l) gi[l] = hm_invmod((u64)bt.gap % mods[l], mods[l]);
      ew1(EW_SCALE, tl, tl, &gi);
      for (u64 gel : bt.trace_gal) {
        Ciphertext r = apply_galois(t, gel);
        ew(EW_ADD, tl, tl, lsq(r.poly, 0, 2, L - 1));
      }
    }
    // CoeffsToSlots
    Ciphertext z = std::move(t);
    for (LinTrans& T : bt.cts) z = lt_rescale(T, z);
    Ciphertext zc = apply_galois(z, 2 * (u64)N - 1);
    Ciphertext y;
    if (bt.gap > 1) {
      // packed real | imaginary parts: z + conj z
      Ciphertext u = new_ct(z.level, B, z.scale);
      ew(EW_ADD, lsq(u.poly, 0, 2, z.level), lsq(z.poly, 0, 2, z.level), lsq(zc.poly, 0, 2, z.level));
      y = eval_mod(bt, u);
    } else {
      // real and imaginary parts: z + conj z, -i (z - conj z)
      Ciphertext re = new_ct(z.level, B, z.scale), im = new_ct(z.level, B, z.scale);
      ew(EW_ADD, lsq(re.poly, 0, 2, z.level), lsq(z.poly, 0, 2, z.level), lsq(zc.poly, 0, 2, z.level));
      ew(EW_SUB, lsq(im.poly, 0, 2, z.level), lsq(zc.poly, 0, 2, z.level), lsq(z.poly, 0, 2, z.level));
      im = mul_i(bt, im);  // (conj z - z) i = -i (z - conj z)
      Ciphertext yr = eval_mod(bt, re), yi = eval_mod(bt, im);
      y = mul_i(bt, yi);
      ew(EW_ADD, lsq(y.poly, 0, 2, y.level), lsq(y.poly, 0, 2, y.level), lsq(yr.poly, 0, 2, y.level));
    }
    // SlotsToCoeffs
    for (LinTrans& T : bt.stc) y = lt_rescale(T, y);
    return y;
  }

  // bootstrapper.go:19-58: one circuit per slot count (made once); logPs
  // empty = the scheme's own P bit sizes
  void new_bootstrapper(std::vector<int> logPs, int ns) {
    typedef Bootstrapper BT;
    if (ci) throw std::runtime_error("bootstrapping needs the Standard ring (Lattigo has no ConjugateInvariant bootstrapper)");
    if (ns < 2 || ns > N / 2 || (ns & (ns - 1)))
      throw std::runtime_error("slots must be a power of two in [2, " + std::to_string(N / 2) + "]");
    if (btps.count(ns)) return;
    if (!have_sk) throw std::runtime_error("bootstrapping keys need the secret key");
    if (logPs.empty()) logPs = logP_bits;
    for (int b : logPs)
      if (b < 20 || b > 61) throw std::runtime_error("bootstrapping P primes must be 20..61 bits");
    auto it = btp_ctx.find(logPs);
    if (it == btp_ctx.end()) {
      // the bootstrapping chain: the residual Q, then SlotsToCoeffs 3 x 39-bit, EvalMod
      // depth(poly) + r x 60-bit, CoeffsToSlots 4 x 56-bit (bottom to top), so the refreshed
      // ciphertext comes out at the residual chain's top level; P from logPs.  New primes skip
      // every prime of the scheme.
      std::vector<int> ext(BT::kStC, BT::kStCBits);
      ext.insert(ext.end(), BT::kDepthPoly + BT::kR, BT::kModBits);
      ext.insert(ext.end(), BT::kCtS, BT::kCtSBits);
      std::vector<int> bits = ext;
      bits.insert(bits.end(), logPs.begin(), logPs.end());
      const std::vector<u64> fresh = gen_moduli_excluding(logN, bits, mods);
      std::vector<u64> m(mods.begin(), mods.begin() + L);
      m.insert(m.end(), fresh.begin(), fresh.end());
      std::vector<int> qb = logQ_bits;
      qb.insert(qb.end(), ext.begin(), ext.end());
      if ((int)m.size() > ORION_MAXMOD || (int)m.size() > ORION_MAXLIMB)
        throw std::runtime_error("bootstrapping chain too long");
      HIPCHK(hipStreamSynchronize(stream));
      std::unique_ptr<Context> bc(new Context());
      bc->stream = stream;  // shared, not owned
      bc->prng = Prng(prng.next());
      bc->init_moduli(logN, m, qb, logPs, logScale, h, false);
      bc->import_secret(secret_coeffs());
      bc->gen_relin();
      it = btp_ctx.emplace(logPs, std::move(bc)).first;
    }
    btps[ns] = it->second->make_circuit(ns);
  }
  // bootstrapper.go:61-80: a new ciphertext at the residual top level, at the
  // input's scale, times the post-scale N / (2 slots)
  Ciphertext bootstrap(const Ciphertext& in, int ns) {
    auto it = btps.find(ns);
    if (it == btps.end()) throw std::runtime_error("no bootstrapper found for slot count: " + std::to_string(ns));
    Bootstrapper& bt = *it->second;
    const int B = in.poly.B;
    // ScaleDown (Lattigo ScaleDown [U]): F = round(q0 / (2^LogMessageRatio
    // scale)) times the level-0 residues (an integer: no level), F from the
    // input's own scale so the message sits 2^-8 below q0 whatever its scale;
    // SlotsToCoeffs carries the default scale's F (bt.F), so the output scale
    // is scale F / bt.F -- the input scale exactly when it is the default
    const long double fr = roundl((long double)mods[0] / ldexpl(in.scale, Bootstrapper::kLogMsgRatio));
    const u64 F = fr < 1 ? 1 : (u64)fr;
    Poly x = alloc(2, 1, B);
    std::vector<u64> f{F % mods[0]};
    ew1(EW_SCALE, lsq(x, 0, 2, 0), lsq(in.poly, 0, 2, 0), &f);
    Ciphertext o = bt.bc->run_circuit(bt, x, B);
    if (o.level != L - 1) throw std::logic_error("bootstrapping circuit did not end at the residual top level");
    Ciphertext out = new_ct(L - 1, B, in.scale * (long double)F / (long double)bt.F);
    // the residual limbs hold the same primes in both contexts
    const LimbSet ol = lsq(out.poly, 0, 2, L - 1);
    if (bt.gap > 1) {  // post-scale (an integer: no level)
      std::vector<u64> ps(L);
      for (int l = 0; l < L; ++l) ps[l] = (u64)bt.gap % mods[l];
      ew1(EW_SCALE, ol, lsq(o.poly, 0, 2, L - 1), &ps);
    } else {
      copy(ol, lsq(o.poly, 0, 2, L - 1));
    }
    return out;
  }
  void delete_bootstrappers() {
    if (stream) HIPCHK(hipStreamSynchronize(stream));
    btps.clear();
    btp_ctx.clear();
  }
};

// ---------------------------------------------------------------------------
// the scheme's contexts: [0] the scheme's own, [1..] its pipelines
// ---------------------------------------------------------------------------
// A pipeline is a context on the scheme's chain that shares the scheme's keys
// and reads the scheme's compiled objects (plaintexts, linear transforms,
// polynomials), with its own HIP stream, buffer pool and handle range.  Each
// thread acts on one context: the thread that made the scheme on the scheme's,
// and, once OrionHipThreadPipelines(n > 1) is set (or ORION_THREAD_PIPELINES=n
// is in the environment), every other thread on a pipeline of its own, made at
// its first call (up to n contexts; further threads share them round-robin).
// So several threads each running the unchanged frontend's `net(ct)` over their
// own ciphertexts run their kernels concurrently on the GPU, each call holding
// only its own context's lock.  Handles are unique across the contexts; calls
// that only name a handle (deletes, metadata) go to the handle's context.
//
// Locks: g_reg (shared by every call, exclusive for NewScheme/DeleteScheme);
// a context's mu for a call acting on it; a thread holding a pipeline's mu may
// take the scheme's (keys, bootstrapping), never the other way round; the
// handle pools' and device pools' locks are leaves.
static std::unique_ptr<Context> g_slot[kMaxCtx];
static std::atomic<int> g_nctx{0};
static std::shared_mutex g_reg;
static std::mutex g_create_mu;
static std::atomic<unsigned long long> g_scheme_gen{1};
static std::atomic<int> g_thread_pipes{getenv("ORION_THREAD_PIPELINES") ? atoi(getenv("ORION_THREAD_PIPELINES")) : 0};
static std::atomic<unsigned> g_rr{0};
static std::thread::id g_scheme_thread;
static unsigned long g_seed = 0x0123456789abcdefull;
struct ThreadBind {
  Context* c = nullptr;
  unsigned long long gen = 0;
};
static thread_local ThreadBind t_bind;
static thread_local Context* t_act = nullptr;  // the context the running call acts on
static thread_local int t_depth = 0;           // nesting of C-ABI calls (SubScalar -> AddScalar)
static thread_local int t_dev = -1;            // this thread's HIP device, as last set here

static Context* scheme_ctx() { return g_nctx.load() > 0 ? g_slot[0].get() : nullptr; }
static Context* slot_ctx(int i) { return i >= 0 && i < g_nctx.load() ? g_slot[i].get() : nullptr; }

static Context& ctx() {
  if (!t_act) throw std::runtime_error("scheme not initialised: call NewScheme first");
  return *t_act;
}

// the caller's stream waits for everything queued on context `owner`'s stream
static void wait_on(Context& me, Context& o) {
  if (&me == &o) return;
  hipEvent_t e;
  HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipEventRecord(e, o.stream));
  HIPCHK(hipStreamWaitEvent(me.stream, e, 0));
  HIPCHK(hipEventDestroy(e));  // (released once the wait has completed)
}
// HandlePool hooks: a call reading another context's object orders its stream
// after that object's producer.  A ciphertext (changed by the ops of its
// context) always waits for its context's queued work; a compiled object
// waits only when it is younger than what this context already waited for
// (every object older than a pipeline was complete when it was made)
static void foreign_order(int owner, unsigned long long birth, bool always) {
  Context* me = t_act;
  Context* o = slot_ctx(owner);
  if (!me || !o || o == me) return;
  if (!always && birth < me->synced[owner]) return;
  if (me->capturing)
    throw std::runtime_error("a captured op reads context " + std::to_string(owner) +
                             "'s newer object: capture on the context that owns it, or run the stream once first");
  const unsigned long long stamp = g_birth.load();
  wait_on(*me, *o);
  if (!always) me->synced[owner] = stamp;
}
static HandlePool<Ciphertext>* res_cts(int i) { Context* c = slot_ctx(i); return c ? &c->cts : nullptr; }
static HandlePool<Plaintext>* res_pts(int i) { Context* c = slot_ctx(i); return c ? &c->pts : nullptr; }
static HandlePool<LinTrans>* res_lts(int i) { Context* c = slot_ctx(i); return c ? &c->lts : nullptr; }
static HandlePool<Context::PolyFn>* res_polys(int i) { Context* c = slot_ctx(i); return c ? &c->polys : nullptr; }
static const bool g_hooks_set = [] {
  HandlePool<Ciphertext>::resolver() = res_cts;
  HandlePool<Plaintext>::resolver() = res_pts;
  HandlePool<LinTrans>::resolver() = res_lts;
  HandlePool<Context::PolyFn>::resolver() = res_polys;
  HandlePool<Ciphertext>::hook() = [](int o, unsigned long long b) { foreign_order(o, b, true); };
  HandlePool<Plaintext>::hook() = [](int o, unsigned long long b) { foreign_order(o, b, false); };
  HandlePool<LinTrans>::hook() = [](int o, unsigned long long b) { foreign_order(o, b, false); };
  HandlePool<Context::PolyFn>::hook() = [](int o, unsigned long long b) { foreign_order(o, b, false); };
  HandlePool<Ciphertext>::check() = [](const Ciphertext& c) {
    if (!c.poison.empty()) throw std::runtime_error(c.poison);
  };
  HandlePool<Ciphertext>::hold() = [](const Ciphertext& c) {
    if (t_act && t_act->capturing && c.poly.buf) t_act->capture_holds.push_back(c.poly.buf);
  };
  HandlePool<Plaintext>::hold() = [](const Plaintext& p) {
    if (t_act && t_act->capturing && p.poly.buf) t_act->capture_holds.push_back(p.poly.buf);
  };
  HandlePool<LinTrans>::hold() = [](const LinTrans& t) {
    if (!t_act || !t_act->capturing) return;
    for (auto& kv : t.diags)
      if (kv.second.poly.buf) t_act->capture_holds.push_back(kv.second.poly.buf);
    for (auto& kv : t.sdiags)
      if (kv.second.buf) t_act->capture_holds.push_back(kv.second.buf);
    if (t.plan) t_act->capture_holds.push_back(t.plan);
  };
  return true;
}();

// a new pipeline context (the caller holds no context lock)
static Context* create_pipeline() {
  std::lock_guard<std::mutex> lk(g_create_mu);
  Context* s = scheme_ctx();
  if (!s) throw std::runtime_error("scheme not initialised: call NewScheme first");
  const int idx = g_nctx.load();
  if (idx >= kMaxCtx) throw std::runtime_error("too many pipelines (" + std::to_string(kMaxCtx - 1) + " at most)");
  std::lock_guard<std::recursive_mutex> sl(s->mu);  // the scheme's keys and transforms are read
  if (t_dev != s->dev) {
    HIPCHK(hipSetDevice(s->dev));
    t_dev = s->dev;
  }
  // the scheme's transforms get their device plans now, so a pipeline only
  // reads them; then every object born so far is complete once the queued
  // work of every context has run
  s->build_dirty_plans();
  const unsigned long long stamp = g_birth.load();
  for (int i = 0; i < idx; ++i) HIPCHK(hipStreamSynchronize(g_slot[i]->stream));
  std::unique_ptr<Context> p(new Context());
  p->index = idx;
  p->dev = s->dev;
  p->prng = Prng(g_seed ^ (0x9e3779b97f4a7c15ull * (u64)idx));
  p->init_moduli(s->logN, s->mods, s->logQ_bits, s->logP_bits, s->logScale, s->h, s->ci);
  p->adopt_keys(*s);
  p->seed_encryption(g_seed + 0x9e3779b97f4a7c15ull * (u64)idx);
  const int base = idx << kCtxShift;
  p->pts.set_base(base), p->cts.set_base(base), p->lts.set_base(base), p->polys.set_base(base);
  p->next_graph = base;
  for (int j = 0; j < kMaxCtx; ++j) p->synced[j] = stamp;
  Context* r = p.get();
  g_slot[idx] = std::move(p);
  g_nctx.store(idx + 1);
  return r;
}

// the context the calling thread acts on (create: a thread's first call may
// make its pipeline); nullptr without a scheme
static Context* thread_ctx(bool create) {
  Context* s = scheme_ctx();
  if (!s) return nullptr;
  const unsigned long long gen = g_scheme_gen.load();
  if (t_bind.c && t_bind.gen == gen) return t_bind.c;
  const int n = g_thread_pipes.load();
  if (n <= 1 || std::this_thread::get_id() == g_scheme_thread) return s;
  if (!create) return s;
  Context* c = nullptr;
  if (g_nctx.load() < n) {
    c = create_pipeline();
  } else {
    const int np = g_nctx.load() - 1;
    c = np > 0 ? g_slot[1 + (int)(g_rr.fetch_add(1) % (unsigned)np)].get() : s;
  }
  t_bind = ThreadBind{c, gen};
  return c;
}
// the context of a handle (deletes and metadata go to the handle's own
// context, whichever thread asks)
static Context* handle_ctx(int id) {
  Context* c = id >= 0 ? slot_ctx(id >> kCtxShift) : nullptr;
  return c ? c : thread_ctx(false);
}

// one C-ABI call: the registry lock (outermost call only), the lock of the
// context it acts on, and that context as the thread's acting one
struct CallScope {
  std::shared_lock<std::shared_mutex> rl;
  std::unique_lock<std::recursive_mutex> cl;
  Context* saved;
  CallScope(bool reg = true) : saved(t_act) {
    if (t_depth++ == 0 && reg) rl = std::shared_lock<std::shared_mutex>(g_reg);
  }
  void act(Context* c) {
    if (!c) return;
    cl = std::unique_lock<std::recursive_mutex>(c->mu);
    t_act = c;
    if (t_dev != c->dev) {
      HIPCHK(hipSetDevice(c->dev));
      t_dev = c->dev;
    }
  }
  ~CallScope() {
    t_act = saved;
    --t_depth;
  }
};

}  // namespace orion

using namespace orion;

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
// C-ABI calls that only enqueue device work (or read host metadata) may be
// recorded into a graph; every other call is refused while a capture is open
static bool capture_ok(const char* fn) {
  static const std::set<std::string> ok = {
      "Negate", "Rotate", "RotateNew", "OrionHipRotateAdd", "Rescale", "RescaleNew", "ModDropCiphertext", "AddScalar", "AddScalarNew",
      "SubScalar", "SubScalarNew", "MulScalarInt", "MulScalarIntNew", "MulScalarFloat", "MulScalarFloatNew",
      "AddPlaintext", "AddPlaintextNew", "SubPlaintext", "SubPlaintextNew", "MulPlaintext", "MulPlaintextNew",
      "AddCiphertext", "AddCiphertextNew", "SubCiphertext", "SubCiphertextNew", "MulRelinCiphertext",
      "MulRelinCiphertextNew", "EvaluateLinearTransform", "EvaluatePolynomial", "CloneCiphertext",
      "DeleteCiphertext", "DeletePlaintext", "SetCiphertextScale", "SetPlaintextScale", "GetCiphertextScale",
      "GetPlaintextScale", "GetCiphertextScaleF", "GetCiphertextLevel", "GetPlaintextLevel", "GetCiphertextSlots",
      "GetPlaintextSlots", "GetCiphertextDegree", "GetCiphertextBatch", "GetPlaintextBatch", "GetLiveCiphertexts",
      "GetLivePlaintexts", "GetModuliChain", "GaloisElement", "OrionHipGraphEnd", "OrionHipGetStream",
      "OrionHipCurrentPipeline"};
  return ok.count(fn) != 0;
}
// debugging switch ORION_DEBUG_SYNC=1: drain the library stream at the start
// of every C-ABI call (separates an ordering race from an arithmetic fault)
static const bool g_debug_sync = getenv("ORION_DEBUG_SYNC") && atoi(getenv("ORION_DEBUG_SYNC")) != 0;
static void capture_guard(const char* fn) {
  Context* c = t_act;
  if (c && c->capturing && !capture_ok(fn))
    throw std::runtime_error(std::string(fn) + " is not allowed while capturing a graph");
  if (g_debug_sync && c && !c->capturing && c->stream) (void)hipStreamSynchronize(c->stream);
}
static int ct_ct_op(int i0, int i1, int op, bool inplace);
// runs a deferred rotation (and the addition recorded after it) exactly as
// the op-by-op calls would have (Context::Deferred).  If it fails, the
// ciphertexts it should have written are poisoned: every later use of x
// (which the AddCiphertext already reported as done) or r fails loudly with
// this error, instead of reading a buffer that was never written
static void poison_deferred(Context& c, const Context::Deferred& d, const char* what) {
  const std::string msg = std::string("a deferred rotation by ") + std::to_string(d.k) + " failed (" + what +
                          "): this ciphertext was never written";
  for (int id : {d.r, d.kind == 2 ? d.x : -1}) {
    if (id < 0) continue;
    try {
      c.cts.get(id).poison = msg;
    } catch (const std::exception&) {
    }
  }
}
static void defer_flush() {
  if (!t_act || !t_act->dfr.kind) return;
  Context& c = *t_act;
  const Context::Deferred d = c.dfr;
  c.dfr = Context::Deferred();
  try {
    c.rotate_into(c.cts.get(d.x), d.k, c.cts.get(d.r));
    if (d.kind == 2) ct_ct_op(d.x, d.r, EW_ADD, true);
  } catch (const std::exception& e) {
    poison_deferred(c, d, e.what());
    throw;
  }
}
// C-ABI calls that leave a pending rotation pending: host metadata reads
// (the deferred result has its level, scale and batch already), error
// strings, and the calls that match it themselves (AddCiphertext,
// DeleteCiphertext); every other call runs it first
static bool defer_keeps(const char* fn) {
  static const std::set<std::string> keep = {
      "AddCiphertext", "DeleteCiphertext", "DeletePlaintext", "GetCiphertextScale", "GetCiphertextScaleF",
      "GetCiphertextLevel", "GetCiphertextSlots", "GetCiphertextDegree", "GetCiphertextBatch", "GetPlaintextScale",
      "GetPlaintextLevel", "GetPlaintextSlots", "GetPlaintextBatch", "GetLiveCiphertexts", "GetLivePlaintexts",
      "GetModuliChain", "GaloisElement", "OrionHipPeerSelect", "OrionHipPeerCount", "OrionHipGetStream",
      "OrionHipCurrentPipeline"};
  return keep.count(fn) != 0;
}
static void defer_gate(const char* fn) {
  if (!t_act || !t_act->dfr.kind) return;
  if (!defer_keeps(fn)) defer_flush();
}
// a call acting on the calling thread's context
#define API_BEGIN         \
  CallScope cs_;          \
  try {                   \
    cs_.act(thread_ctx(true)); \
    capture_guard(__func__); \
    defer_gate(__func__);
// a call acting on the context of handle `id`
#define API_BEGIN_HANDLE(id) \
  CallScope cs_;             \
  try {                      \
    cs_.act(handle_ctx(id)); \
    capture_guard(__func__); \
    defer_gate(__func__);
// a call acting on no context (or on several, one at a time)
#define API_BEGIN_NOCTX \
  CallScope cs_;        \
  try {
// NewScheme / DeleteScheme: every other call is kept out
#define API_BEGIN_EXCL                                \
  std::unique_lock<std::shared_mutex> xl_(g_reg);     \
  CallScope cs_(false);                               \
  try {
// (a failed call's HIP error is read off here, so that it is reported once,
// by this call, and not again by the next call's launch checks)
#define API_END(errval)          \
  }                              \
  catch (const std::exception& e) { \
    g_last_error = e.what();     \
    (void)hipGetLastError();     \
    return errval;               \
  }
#define API_END_VOID                \
  }                                 \
  catch (const std::exception& e) { \
    g_last_error = e.what();        \
    (void)hipGetLastError();        \
  }

template <class T, class U>
static U* to_c_array(const std::vector<T>& v, unsigned long* len) {
  *len = v.size();
  if (v.empty()) return nullptr;
  U* p = (U*)malloc(sizeof(U) * v.size());
  for (size_t i = 0; i < v.size(); ++i) p[i] = (U)v[i];
  return p;
}

extern "C" {

const char* OrionHipLastError(void) { return g_last_error.c_str(); }
void OrionHipClearError(void) { g_last_error.clear(); }

static hipStream_t g_user_stream = nullptr;

int OrionHipSetDevice(int device) {
  API_BEGIN_NOCTX
  HIPCHK(hipSetDevice(device));
  t_dev = device;
  return 0;
  API_END(-1)
}

void OrionHipSetSeed(unsigned long seed) {
  API_BEGIN
  g_seed = seed;
  if (t_act) {
    t_act->prng = Prng(seed);
    t_act->seed_encryption(seed);
  }
  API_END_VOID
}

void OrionHipSetStream(void* s) {
  API_BEGIN
  Context* c = t_act;
  if (!c || c->index == 0) g_user_stream = (hipStream_t)s;
  if (c) {
    // the buffer pool hands freed buffers out again with no stream tracking:
    // drain the old stream so no kernel still reading or writing a pooled
    // buffer overlaps the first launches on the new one
    if (c->stream) HIPCHK(hipStreamSynchronize(c->stream));
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    c->own_stream = false;
    c->stream = (hipStream_t)s;
    if (!s) {
      HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      c->own_stream = true;
    }
    for (auto& kv : c->btp_ctx) kv.second->stream = c->stream;
  }
  API_END_VOID
}

// the calling thread's context's stream (a thread's first call binds it to
// its pipeline when thread pipelines are on)
void* OrionHipGetStream(void) {
  API_BEGIN
  return t_act ? (void*)t_act->stream : nullptr;
  API_END(nullptr)
}

int OrionHipSynchronize(void) {  // every context's stream (the pipelines' included)
  API_BEGIN_NOCTX
  if (!scheme_ctx()) throw std::runtime_error("scheme not initialised: call NewScheme first");
  for (int i = 0; i < g_nctx.load(); ++i) HIPCHK(hipStreamSynchronize(g_slot[i]->stream));
  return 0;
  API_END(-1)
}

// ---- hipGraph capture of op streams (see Context::graph_begin) ----
int OrionHipGraphBegin(void) {
  API_BEGIN
  ctx().graph_begin();
  return 0;
  API_END(-1)
}
int OrionHipGraphEnd(void) {
  API_BEGIN
  return ctx().graph_end();
  API_END(-1)
}
int OrionHipGraphLaunch(int graph) {  // on the stream of the context that captured it
  API_BEGIN_HANDLE(graph)
  ctx().graph_launch(graph);
  return 0;
  API_END(-1)
}
void OrionHipGraphDestroy(int graph) {
  API_BEGIN_HANDLE(graph)
  ctx().graph_destroy(graph);
  API_END_VOID
}

int OrionHipLogN(void) { return scheme_ctx() ? scheme_ctx()->logN : -1; }
int OrionHipNumQ(void) { return scheme_ctx() ? scheme_ctx()->L : -1; }
int OrionHipNumP(void) { return scheme_ctx() ? scheme_ctx()->K : -1; }
unsigned long OrionHipModulus(int i) {
  Context* s = scheme_ctx();
  return (s && i >= 0 && i < (int)s->mods.size()) ? s->mods[i] : 0;
}

void NewScheme(int logN, int* logQ, int lenQ, int* logP, int lenP, int logScale, int h, char* ringType,
               char* keysPath, char* ioMode) {
  API_BEGIN_EXCL
  (void)keysPath;
  (void)ioMode;
  std::string rt = ringType ? ringType : "standard";
  for (auto& ch : rt) ch = (char)tolower(ch);
  // scheme.go:50-51: any ring type other than "standard" selects Lattigo's
  // ConjugateInvariant ring Z[X + X^-1]/(X^2N + 1) of degree N (NthRoot 4N,
  // N real slots), held natively: N coefficients per limb, the NTT folds and
  // unfolds around the degree-N transform (ntt.hip, Context::setup).
  const bool ci = rt != "standard";
  if (ci && rt != "conjugateinvariant")
    throw std::runtime_error("unknown ring type '" + rt + "' (standard | conjugateinvariant)");
  // the CI NTT folds/unfolds inside the one-pass kernels (N <= 2^15 per CU)
  if (ci && (logN < 13 || logN > 15))
    throw std::runtime_error("ConjugateInvariant ring: logN must be 13..15 in this build");
  for (int i = g_nctx.load() - 1; i >= 0; --i) g_slot[i].reset();  // pipelines first
  g_nctx.store(0);
  g_scheme_gen.fetch_add(1);
  std::unique_ptr<Context> c(new Context());
  c->index = 0;
  HIPCHK(hipGetDevice(&c->dev));
  t_dev = c->dev;
  c->stream = g_user_stream;
  c->prng = Prng(g_seed);
  c->setup(logN, std::vector<int>(logQ, logQ + lenQ), std::vector<int>(logP, logP + lenP), logScale, h, ci);
  c->seed_encryption(g_seed);
  g_scheme_thread = std::this_thread::get_id();
  t_bind = ThreadBind{c.get(), g_scheme_gen.load()};
  g_slot[0] = std::move(c);
  g_nctx.store(1);
  API_END_VOID
}

void DeleteScheme(void) {
  API_BEGIN_EXCL
  for (int i = g_nctx.load() - 1; i >= 0; --i) g_slot[i].reset();  // pipelines first
  g_nctx.store(0);
  g_scheme_gen.fetch_add(1);
  API_END_VOID
}

// Pipelines (see the registry above).  OrionHipPeerCreate makes one and
// returns its index (the scheme's context is 0) without binding any thread;
// OrionHipPeerSelect binds the calling thread to a context; with
// OrionHipThreadPipelines(n > 1) threads are bound automatically.
int OrionHipPeerCreate(void) {
  API_BEGIN_NOCTX
  return create_pipeline()->index;
  API_END(-1)
}
int OrionHipPeerSelect(int id) {
  API_BEGIN_NOCTX
  Context* c = slot_ctx(id);
  if (!c) throw std::runtime_error("no such pipeline context: " + std::to_string(id));
  t_bind = ThreadBind{c, g_scheme_gen.load()};
  return 0;
  API_END(-1)
}
int OrionHipPeerCount(void) { return g_nctx.load(); }
// n > 1: every thread other than the scheme's gets a pipeline of its own at
// its first call, up to n contexts in all (then round-robin); n <= 1: off.
// Returns the previous setting.
int OrionHipThreadPipelines(int n) { return g_thread_pipes.exchange(n); }
// the index of the calling thread's context (binding it, as any call does)
int OrionHipCurrentPipeline(void) {
  API_BEGIN
  return ctx().index;
  API_END(-1)
}
// ORION_POOL_CAP_BYTES at run time (0: no cap; see DevicePool::alloc);
// returns the previous cap
double OrionHipPoolCap(double bytes) {
  std::lock_guard<std::recursive_mutex> lk(DevicePool::mu());
  const double prev = DevicePool::cap_bytes();
  DevicePool::cap_ref() = bytes;
  return prev;
}
int OrionHipPoolStats(double* out, int n) {
  std::lock_guard<std::recursive_mutex> lk(DevicePool::mu());
  double cached = 0;
  for (DevicePool* q : DevicePool::registry()) cached += (double)q->cached();
  const double v[5] = {DevicePool::stats()[0], DevicePool::stats()[1], DevicePool::stats()[2], DevicePool::stats()[3],
                       cached};
  for (int i = 0; i < n && i < 5; ++i) out[i] = v[i];
  return 5;
}
int OrionHipStreamWaitPeer(int peer) {
  API_BEGIN
  Context* p = slot_ctx(peer);
  if (!p) throw std::runtime_error("no such pipeline context: " + std::to_string(peer));
  wait_on(ctx(), *p);
  return 0;
  API_END(-1)
}

void FreeCArray(void* p) { free(p); }

void DeletePlaintext(int id) {
  API_BEGIN_HANDLE(id)
  ctx().pts.del(id);
  API_END_VOID
}
void DeleteCiphertext(int id) {
  API_BEGIN_HANDLE(id)
  Context& c = ctx();
  const Context::Deferred d = c.dfr;
  if (d.kind && id == d.r) {
    c.dfr = Context::Deferred();
    // the rotation dies unread: kind 1 needs no work at all; kind 2 is
    // x += Rotate(x, k) with the addition in the key switch's store.  The
    // handle goes away whatever happens; if the key switch fails, x (which
    // the AddCiphertext reported as done) is poisoned
    if (d.kind == 2) {
      try {
        c.rotate_add_inplace(c.cts.get(d.x), d.k);
      } catch (const std::exception& e) {
        poison_deferred(c, d, e.what());
        c.cts.del(id);
        throw;
      }
    }
  } else if (d.kind && id == d.x) {
    try {
      defer_flush();
    } catch (const std::exception&) {
      c.cts.del(id);
      throw;
    }
  }
  c.cts.del(id);
  API_END_VOID
}

static unsigned long scale_u64(long double s) {
  if (s >= 18446744073709551615.0L) return ~0ul;
  return (unsigned long)s;
}
unsigned long GetPlaintextScale(int id) {
  API_BEGIN_HANDLE(id)
  return scale_u64(ctx().pts.get(id).scale);
  API_END(0)
}
unsigned long GetCiphertextScale(int id) {
  API_BEGIN_HANDLE(id)
  return scale_u64(ctx().cts.get(id).scale);
  API_END(0)
}
double GetCiphertextScaleF(int id) {
  API_BEGIN_HANDLE(id)
  return (double)ctx().cts.get(id).scale;
  API_END(0)
}
void SetPlaintextScale(int id, unsigned long s) {
  API_BEGIN_HANDLE(id)
  ctx().pts.get(id).scale = (long double)s;
  API_END_VOID
}
void SetCiphertextScale(int id, unsigned long s) {
  API_BEGIN_HANDLE(id)
  ctx().cts.get(id).scale = (long double)s;
  API_END_VOID
}
int GetPlaintextLevel(int id) {
  API_BEGIN_HANDLE(id)
  return ctx().pts.get(id).level;
  API_END(-1)
}
int GetCiphertextLevel(int id) {
  API_BEGIN_HANDLE(id)
  return ctx().cts.get(id).level;
  API_END(-1)
}
int GetPlaintextSlots(int id) {
  API_BEGIN_HANDLE(id)
  ctx().pts.get(id);
  return ctx().slots;
  API_END(-1)
}
int GetCiphertextSlots(int id) {
  API_BEGIN_HANDLE(id)
  ctx().cts.get(id);
  return ctx().slots;
  API_END(-1)
}
int GetCiphertextDegree(int id) {
  API_BEGIN_HANDLE(id)
  ctx().cts.get(id);
  return 1;
  API_END(-1)
}
int GetCiphertextBatch(int id) {
  API_BEGIN_HANDLE(id)
  return ctx().cts.get(id).poly.B;
  API_END(-1)
}
int GetPlaintextBatch(int id) {
  API_BEGIN_HANDLE(id)
  return ctx().pts.get(id).poly.B;
  API_END(-1)
}
ArrayResultUInt64 GetModuliChain(void) {
  ArrayResultUInt64 r{nullptr, 0};
  API_BEGIN
  std::vector<u64> q(ctx().mods.begin(), ctx().mods.begin() + ctx().L);
  r.Data = to_c_array<u64, unsigned long>(q, &r.Length);
  return r;
  API_END(r)
}
ArrayResultInt GetLivePlaintexts(void) {
  ArrayResultInt r{nullptr, 0};
  API_BEGIN
  r.Data = to_c_array<int, int>(ctx().pts.live(), &r.Length);
  return r;
  API_END(r)
}
ArrayResultInt GetLiveCiphertexts(void) {
  ArrayResultInt r{nullptr, 0};
  API_BEGIN
  r.Data = to_c_array<int, int>(ctx().cts.live(), &r.Length);
  return r;
  API_END(r)
}
int CloneCiphertext(int id) {
  API_BEGIN
  Context& c = ctx();
  return c.cts.add(c.clone(c.cts.get(id)));
  API_END(-1)
}

// ---- keys ----
void NewKeyGenerator(void) {}
void GenerateSecretKey(void) {
  API_BEGIN
  ctx().gen_secret();
  API_END_VOID
}
void GeneratePublicKey(void) {
  API_BEGIN
  ctx().gen_public();
  API_END_VOID
}
void GenerateRelinearizationKey(void) {
  API_BEGIN
  ctx().gen_relin();
  API_END_VOID
}
void GenerateEvaluationKeys(void) {}

// ---- Lattigo v6 wire formats (wire.h): rlwe.SecretKey = ringqp.Poly ----
static std::vector<u64> mods_of(const Context& c, int nq, bool with_p) {
  std::vector<u64> m(c.mods.begin(), c.mods.begin() + nq);
  if (with_p) m.insert(m.end(), c.mods.begin() + c.L, c.mods.begin() + c.L + c.K);
  return m;
}
// ringqp.Poly of a [nq + K][N] host block: ring.Poly Q (nq limbs), ring.Poly P (K limbs)
static void put_qp(std::vector<char>& b, const Context& c, const u64* data, int nq) {
  wire::put_poly(b, data, mods_of(c, nq, false), c.N);
  std::vector<u64> pm(c.mods.begin() + c.L, c.mods.begin() + c.L + c.K);
  wire::put_poly(b, data + (size_t)nq * c.N, pm, c.N);
}
static void get_qp(wire::Reader& rd, const Context& c, u64* out, int nq, const char* what) {
  rd.get_poly(out, mods_of(c, nq, false), c.N, what);
  std::vector<u64> pm(c.mods.begin() + c.L, c.mods.begin() + c.L + c.K);
  rd.get_poly(out + (size_t)nq * c.N, pm, c.N, what);
}
static ArrayResultByte to_bytes(const std::vector<char>& v) {
  ArrayResultByte r{nullptr, 0};
  r.Data = to_c_array<char, char>(v, &r.Length);
  return r;
}
// rlwe.GaloisKey: GaloisElement, NthRoot, GadgetCiphertext{BaseTwoDecomposition 0,
// Value: beta x 1 VectorQP (k0, k1)} of a [beta][2][level+1+K][N] host key made
// for `level` (Lattigo's key at LevelQ = level: beta rows, level+1 Q limbs)
static std::vector<char> galois_key_bytes(const Context& c, u64 galEl, const std::vector<u64>& key, int level) {
  std::vector<char> b;
  const int beta = (level + 1 + c.K - 1) / c.K;
  const size_t qp = (size_t)(level + 1 + c.K) * c.N;
  b.reserve(40 + (size_t)beta * (16 + 2 * (wire::poly_bytes(level + 1, c.N) + wire::poly_bytes(c.K, c.N))));
  wire::put_u64(b, galEl);
  wire::put_u64(b, c.nthroot);  // NthRoot
  wire::put_u64(b, 0);             // BaseTwoDecomposition
  wire::put_u64(b, (u64)beta);     // Matrix rows
  for (int i = 0; i < beta; ++i) {
    wire::put_u64(b, 1);  // one column (no power-of-two decomposition)
    wire::put_u64(b, 2);  // VectorQP length
    for (int k = 0; k < 2; ++k) put_qp(b, c, key.data() + (2 * (size_t)i + k) * qp, level + 1);
  }
  return b;
}

ArrayResultByte SerializeSecretKey(void) {
  ArrayResultByte r{nullptr, 0};
  API_BEGIN
  Context& c = ctx();
  if (!c.have_sk) throw std::runtime_error("secret key not generated");
  std::vector<u64> host;
  c.download(c.sk, host);
  std::vector<char> bytes;
  put_qp(bytes, c, host.data(), c.L);
  return to_bytes(bytes);
  API_END(r)
}
void LoadSecretKey(char* data, unsigned long len) {
  API_BEGIN
  Context& c = ctx();
  if (!data) throw std::runtime_error("null secret key data");
  wire::Reader rd(data, len);
  std::vector<u64> host((size_t)(c.L + c.K) * c.N);
  get_qp(rd, c, host.data(), c.L, "secret key");
  if (rd.left()) throw std::runtime_error("secret key blob has trailing bytes");
  c.sk = c.alloc(1, c.L + c.K, 1);
  c.upload(c.sk, host);
  c.have_sk = true;
  API_END_VOID
}

// ---- encoder / encryptor ----
void NewEncoder(void) {}
int Encode(float* values, int n, int level, unsigned long scale) {
  API_BEGIN
  Context& c = ctx();
  if (level < 0 || level >= c.L) throw std::runtime_error("invalid level");
  return c.pts.add(c.encode(values, n, 1, level, (long double)scale, false));
  API_END(-1)
}
int EncodeBatch(float* values, int n, int B, int level, unsigned long scale) {
  API_BEGIN
  Context& c = ctx();
  if (level < 0 || level >= c.L || B < 1) throw std::runtime_error("invalid level/batch");
  return c.pts.add(c.encode(values, n, B, level, (long double)scale, false));
  API_END(-1)
}
int EncodeBatchDevice(const float* dvalues, int n, int B, int level, double scale) {
  API_BEGIN
  Context& c = ctx();
  if (level < 0 || level >= c.L || B < 1 || !dvalues) throw std::runtime_error("invalid level/batch/pointer");
  return c.pts.add(c.encode_dev(dvalues, n, B, level, (long double)scale, false));
  API_END(-1)
}
int DecodeDevice(int pt, double* dout) {
  API_BEGIN
  Context& c = ctx();
  if (!dout) throw std::runtime_error("null output pointer");
  c.decode_dev(c.pts.get(pt), dout);
  return 0;
  API_END(-1)
}
int DecodeF64(int pt, double* out, unsigned long n) {
  API_BEGIN
  Context& c = ctx();
  const Plaintext& p = c.pts.get(pt);
  if (n < (unsigned long)p.poly.B * (c.slots)) throw std::runtime_error("output buffer too small");
  std::vector<double> v = c.decode(p);
  memcpy(out, v.data(), v.size() * sizeof(double));
  return 0;
  API_END(-1)
}
ArrayResultFloat Decode(int id) {
  ArrayResultFloat r{nullptr, 0};
  API_BEGIN
  Context& c = ctx();
  std::vector<double> v = c.decode(c.pts.get(id));
  r.Data = to_c_array<double, float>(v, &r.Length);
  return r;
  API_END(r)
}
void NewEncryptor(void) {}
void NewDecryptor(void) {}
int Encrypt(int pt) {
  API_BEGIN
  Context& c = ctx();
  return c.cts.add(c.encrypt(c.pts.get(pt)));
  API_END(-1)
}
int Decrypt(int ct) {
  API_BEGIN
  Context& c = ctx();
  return c.pts.add(c.decrypt(c.cts.get(ct)));
  API_END(-1)
}

// ---- evaluator ----
void NewEvaluator(void) {
  API_BEGIN
  Context& c = ctx();
  for (int i = 1; i < c.slots; i *= 2) c.gen_galois(c.galois_element(i), c.L - 1);  // evaluator.go:25-31
  API_END_VOID
}
void AddRotationKey(int k) {
  API_BEGIN
  Context& c = ctx();
  c.gen_galois(c.galois_element(k), c.L - 1);
  API_END_VOID
}
unsigned long GaloisElement(int k) {
  API_BEGIN
  return ctx().galois_element(k);
  API_END(0)
}

int Negate(int id) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.cts.get(id);
  Ciphertext o = c.new_ct(a.level, a.poly.B, a.scale);
  c.ew1(EW_NEG, c.lsq(o.poly, 0, 2, a.level), c.lsq(a.poly, 0, 2, a.level));
  return c.cts.add(std::move(o));
  API_END(-1)
}
int Rotate(int id, int k) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.inplace_ct(id, false);  // the rotation replaces a (buffer and copy-on-write share)
  a = c.rotate(a, k);
  return id;
  API_END(-1)
}
int RotateNew(int id, int k) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.cts.get(id);
  if (!c.defer_on) return c.cts.add(c.rotate(a, k));
  // deferred (Context::Deferred): the key is made (or checked) now, so a
  // missing key fails here as in the op-by-op path; r gets no buffer yet
  c.galois_key(c.galois_element(k), a.level);
  Ciphertext r;
  r.level = a.level;
  r.scale = a.scale;
  r.poly.B = a.poly.B;
  const int rid = c.cts.add(std::move(r));
  c.dfr = Context::Deferred{1, id, rid, k};
  return rid;
  API_END(-1)
}
int OrionHipRotateAdd(int id, int k) {
  API_BEGIN
  Context& c = ctx();
  c.rotate_add_inplace(c.inplace_ct(id), k);
  return id;
  API_END(-1)
}
int Rescale(int id) {
  API_BEGIN
  Context& c = ctx();
  c.rescale_inplace(c.inplace_ct(id));
  return id;
  API_END(-1)
}
int RescaleNew(int id) {  // evaluator.go:92-99: rescales the input in place, returns a copy
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.inplace_ct(id);
  c.rescale_inplace(a);
  return c.cts.add(c.alias(a));  // copy-on-write: the copy is made only if both are later written
  API_END(-1)
}

// evaluator.py:30-41 (the fork's HEonGPU-only mod_drop): drop the top modulus
// in place, scale unchanged; returns the input id
int ModDropCiphertext(int id) {
  API_BEGIN
  Ciphertext& a = ctx().inplace_ct(id);
  if (a.level < 1) throw std::runtime_error("cannot drop the last modulus");
  a.level -= 1;
  return id;
  API_END(-1)
}

static Ciphertext add_scalar(Context& c, const Ciphertext& a, float v, bool inplace_target, Ciphertext* dst) {
  (void)inplace_target;
  long double x = (long double)v * a.scale;
  long double r = x < 0 ? -floorl(-x + 0.5L) : floorl(x + 0.5L);
  std::vector<u64> k = c.const_residues(r, a.level);
  Ciphertext o = dst ? Ciphertext() : c.new_ct(a.level, a.poly.B, a.scale);
  Ciphertext& out = dst ? *dst : o;
  c.ew1(EW_ADDC, c.lsq(out.poly, 0, 1, a.level), c.lsq(a.poly, 0, 1, a.level), &k);
  if (!dst) c.copy(c.lsq(out.poly, 1, 1, a.level), c.lsq(a.poly, 1, 1, a.level));
  return o;
}
int AddScalar(int id, float v) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.inplace_ct(id);
  add_scalar(c, a, v, true, &a);
  return id;
  API_END(-1)
}
int AddScalarNew(int id, float v) {
  API_BEGIN
  Context& c = ctx();
  return c.cts.add(add_scalar(c, c.cts.get(id), v, false, nullptr));
  API_END(-1)
}
int SubScalar(int id, float v) { return AddScalar(id, -v); }
int SubScalarNew(int id, float v) { return AddScalarNew(id, -v); }

static void mul_const(Context& c, const Ciphertext& a, Ciphertext& out, const std::vector<u64>& k) {
  c.ew1(EW_SCALE, c.lsq(out.poly, 0, 2, a.level), c.lsq(a.poly, 0, 2, a.level), &k);
}
int MulScalarInt(int id, int v) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.inplace_ct(id);
  mul_const(c, a, a, c.const_residues((long double)v, a.level));
  return id;
  API_END(-1)
}
int MulScalarIntNew(int id, int v) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.cts.get(id);
  Ciphertext o = c.new_ct(a.level, a.poly.B, a.scale);
  mul_const(c, a, o, c.const_residues((long double)v, a.level));
  return c.cts.add(std::move(o));
  API_END(-1)
}
// non-integral constants are scaled by q_level (Lattigo getConstantAndScale)
static void mul_float(Context& c, const Ciphertext& a, Ciphertext& out, float v) {
  const double dv = (double)v;
  if (dv == floor(dv)) {
    mul_const(c, a, out, c.const_residues((long double)dv, a.level));
    out.scale = a.scale;
    return;
  }
  const long double ql = (long double)c.mods[a.level];
  long double x = (long double)dv * ql;
  long double r = x < 0 ? -floorl(-x + 0.5L) : floorl(x + 0.5L);
  mul_const(c, a, out, c.const_residues(r, a.level));
  out.scale = a.scale * ql;
}
int MulScalarFloat(int id, float v) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.inplace_ct(id);
  mul_float(c, a, a, v);
  return id;
  API_END(-1)
}
int MulScalarFloatNew(int id, float v) {
  API_BEGIN
  Context& c = ctx();
  Ciphertext& a = c.cts.get(id);
  Ciphertext o = c.new_ct(a.level, a.poly.B, a.scale);
  mul_float(c, a, o, v);
  return c.cts.add(std::move(o));
  API_END(-1)
}

// ct (+/-) pt
static int ct_pt_op(int id, int pid, int op, bool inplace) {
  Context& c = ctx();
  Ciphertext& a = inplace ? c.inplace_ct(id) : c.cts.get(id);
  const Plaintext& p = c.pts.get(pid);
  const int level = std::min(a.level, p.level);
  const int B = c.batch_of(a.poly.B, p.poly.B);
  if (inplace && B != a.poly.B) throw std::runtime_error("in-place op cannot grow the batch");
  Ciphertext o;
  Ciphertext* out = &a;
  if (!inplace) {
    o = c.new_ct(level, B, a.scale);
    out = &o;
  }
  out->level = level;
  c.add_like(*out, a, c.lsq(p.poly, 0, 1, level, B), p.scale, op);
  return inplace ? id : c.cts.add(std::move(o));
}
int AddPlaintext(int id, int pt) {
  API_BEGIN
  return ct_pt_op(id, pt, EW_ADD, true);
  API_END(-1)
}
int AddPlaintextNew(int id, int pt) {
  API_BEGIN
  return ct_pt_op(id, pt, EW_ADD, false);
  API_END(-1)
}
int SubPlaintext(int id, int pt) {
  API_BEGIN
  return ct_pt_op(id, pt, EW_SUB, true);
  API_END(-1)
}
int SubPlaintextNew(int id, int pt) {
  API_BEGIN
  return ct_pt_op(id, pt, EW_SUB, false);
  API_END(-1)
}
static int ct_pt_mul(int id, int pid, bool inplace) {
  Context& c = ctx();
  Ciphertext& a = inplace ? c.inplace_ct(id) : c.cts.get(id);
  const Plaintext& p = c.pts.get(pid);
  const int level = std::min(a.level, p.level);
  const int B = c.batch_of(a.poly.B, p.poly.B);
  if (inplace && B != a.poly.B) throw std::runtime_error("in-place op cannot grow the batch");
  Ciphertext o;
  Ciphertext* out = &a;
  if (!inplace) {
    o = c.new_ct(level, B, a.scale);
    out = &o;
  }
  LimbSet lp = c.lsq(p.poly, 0, 1, level, B);
  lp.ncomp = 2;
  lp.comp_stride = 0;
  c.ew(EW_MUL, c.lsq(out->poly, 0, 2, level), c.lsq(a.poly, 0, 2, level, B), lp);
  out->level = level;
  out->scale = a.scale * p.scale;
  return inplace ? id : c.cts.add(std::move(o));
}
int MulPlaintext(int id, int pt) {
  API_BEGIN
  return ct_pt_mul(id, pt, true);
  API_END(-1)
}
int MulPlaintextNew(int id, int pt) {
  API_BEGIN
  return ct_pt_mul(id, pt, false);
  API_END(-1)
}
static int ct_ct_op(int i0, int i1, int op, bool inplace) {
  Context& c = ctx();
  Ciphertext& a = inplace ? c.inplace_ct(i0) : c.cts.get(i0);
  const Ciphertext& b = c.cts.get(i1);
  const int level = std::min(a.level, b.level);
  const int B = c.batch_of(a.poly.B, b.poly.B);
  if (inplace && B != a.poly.B) throw std::runtime_error("in-place op cannot grow the batch");
  Ciphertext o;
  Ciphertext* out = &a;
  if (!inplace) {
    o = c.new_ct(level, B, a.scale);
    out = &o;
  }
  out->level = level;
  c.add_like(*out, a, c.lsq(b.poly, 0, 2, level, B), b.scale, op);
  return inplace ? i0 : c.cts.add(std::move(o));
}
int AddCiphertext(int a, int b) {
  API_BEGIN
  Context& c = ctx();
  if (c.dfr.kind == 1 && a == c.dfr.x && b == c.dfr.r) {  // x += (pending) Rotate(x, k): record the sum
    c.inplace_ct(a);
    c.dfr.kind = 2;
    return a;
  }
  defer_flush();
  return ct_ct_op(a, b, EW_ADD, true);
  API_END(-1)
}
int AddCiphertextNew(int a, int b) {
  API_BEGIN
  return ct_ct_op(a, b, EW_ADD, false);
  API_END(-1)
}
int SubCiphertext(int a, int b) {
  API_BEGIN
  return ct_ct_op(a, b, EW_SUB, true);
  API_END(-1)
}
int SubCiphertextNew(int a, int b) {
  API_BEGIN
  return ct_ct_op(a, b, EW_SUB, false);
  API_END(-1)
}
int MulRelinCiphertext(int a, int b) {
  API_BEGIN
  Context& c = ctx();
  c.inplace_ct(a, false);  // the product replaces a (buffer and copy-on-write share)
  Ciphertext r = c.mul_relin(c.cts.get(a), c.cts.get(b));
  if (r.poly.B != c.cts.get(a).poly.B) throw std::runtime_error("in-place op cannot grow the batch");
  c.cts.get(a) = std::move(r);
  return a;
  API_END(-1)
}
int MulRelinCiphertextNew(int a, int b) {
  API_BEGIN
  Context& c = ctx();
  return c.cts.add(c.mul_relin(c.cts.get(a), c.cts.get(b)));
  API_END(-1)
}

// ---- linear transforms ----
void NewLinearTransformEvaluator(void) {}

static void bsgs_split(int rot, int slots, int N1, int* giant, int* baby) {
  rot &= (slots - 1);
  *giant = ((rot / N1) * N1) & (slots - 1);
  *baby = rot & (N1 - 1);
}
// Lattigo lintrans FindBestBSGSRatio
static int find_best_n1(const std::vector<int>& idx, int slots, int logMaxRatio) {
  const double maxRatio = (double)(1 << logMaxRatio);
  for (int N1 = 1; N1 < slots; N1 <<= 1) {
    std::set<int> gs, bs;
    for (int d : idx) {
      int gi, bi;
      bsgs_split(d, slots, N1, &gi, &bi);
      gs.insert(gi);
      bs.insert(bi);
    }
    const double r = (double)((int)bs.size() - 1) / (double)((int)gs.size() - 1);
    if (r == maxRatio) return N1;
    if (r > maxRatio) return N1 / 2;
  }
  return 1;
}

int GenerateLinearTransform(int* diagIdx, int nIdx, float* data, int nData, int level, float ratio,
                            char* ioMode) {
  API_BEGIN
  Context& c = ctx();
  // lineartransform.go:79-88: in "load" mode the diagonals were serialised
  // earlier and arrive through LoadPlaintextDiagonal, so none is encoded here
  const bool load = ioMode && std::string(ioMode) == "load";
  const int slots = c.slots;
  if (!load && (long)nIdx * slots != (long)nData) throw std::runtime_error("diagonal data length != nIdx * slots");
  if (level < 0 || level >= c.L) throw std::runtime_error("invalid level");
  LinTrans T;
  T.level = level;
  T.ratio = ratio;
  T.idx.assign(diagIdx, diagIdx + nIdx);
  const int logRatio = (int)log((double)ratio);  // lineartransform.go:67 (natural log)
  if (logRatio < 0) throw std::runtime_error("naive (non-BSGS) linear transforms are not supported");
  T.N1 = find_best_n1(T.idx, slots, logRatio);
  std::set<int> seenb;
  for (int d : T.idx) {
    int gi, bi;
    bsgs_split(d, slots, T.N1, &gi, &bi);
    T.index[gi].push_back(bi);
    if (!seenb.count(bi)) {
      seenb.insert(bi);
      T.babies.push_back(bi);
    }
  }
  for (auto& kv : T.index) {
    std::sort(kv.second.begin(), kv.second.end());
    T.giants.push_back(kv.first);
  }
  for (int r : T.giants)
    if (r) c.key_hint[c.galois_element(r)] = std::max(c.key_hint[c.galois_element(r)], level);
  for (int r : T.babies)
    if (r) c.key_hint[c.galois_element(r)] = std::max(c.key_hint[c.galois_element(r)], level);
  std::vector<float> vec(slots);
  for (int i = 0; i < nIdx && !load; ++i) {
    int gi, bi;
    bsgs_split(diagIdx[i], slots, T.N1, &gi, &bi);
    const float* v = data + (size_t)i * slots;
    for (int s = 0; s < slots; ++s) vec[s] = v[((s - gi) % slots + slots) % slots];  // rotate right by giant
    T.diags[diagIdx[i] & (slots - 1)] = c.encode(vec.data(), slots, 1, level, (long double)c.mods[level], true);
  }
  return c.lts.add(std::move(T));
  API_END(-1)
}

int GetLinearTransformN1(int id) {
  API_BEGIN_HANDLE(id)
  return ctx().lts.get(id).N1;
  API_END(-1)
}

int EvaluateLinearTransform(int tid, int cid) {
  API_BEGIN
  Context& c = ctx();
  LinTrans& T = c.lts.get(tid);
  Context* o = handle_ctx(tid);
  if (T.plan_dirty && o && o != &c) {
    // another context's transform whose plan is not built (its diagonals
    // changed after the pipelines were made): its owner builds it, under its
    // lock -- only a lower-index context may be waited on (lock order)
    if (o->index > c.index) throw std::runtime_error("linear transform " + std::to_string(tid) + " of pipeline " + std::to_string(o->index) + " has no device plan yet: evaluate it there first");
    std::lock_guard<std::recursive_mutex> lk(o->mu);
    if (T.plan_dirty) o->build_plan(T);
  }
  return c.cts.add(c.eval_lt(T, c.cts.get(cid)));
  API_END(-1)
}
void DeleteLinearTransform(int id) {
  API_BEGIN_HANDLE(id)
  ctx().lts.del(id);
  API_END_VOID
}
ArrayResultInt GetLinearTransformRotationKeys(int id) {
  ArrayResultInt r{nullptr, 0};
  API_BEGIN
  Context& c = ctx();
  const LinTrans& T = c.lts.get(id);
  std::vector<int> rots(T.giants.begin(), T.giants.end());
  for (int b : T.babies)
    if (std::find(rots.begin(), rots.end(), b) == rots.end()) rots.push_back(b);
  std::vector<int> gels;
  for (int k : rots) gels.push_back((int)c.galois_element(k));
  r.Data = to_c_array<int, int>(gels, &r.Length);
  return r;
  API_END(r)
}
// keys asked for by a linear transform are made for the highest level of the
// transforms that use them (key_hint); any other element gets a full-chain key
void GenerateLinearTransformRotationKey(int galEl) {
  API_BEGIN
  Context& c = ctx();
  const u64 g = (u64)(unsigned)galEl;
  if (g != 1) c.gen_galois(g, c.hinted_level(g));  // 1 = the identity (zero rotation): no key needed
  API_END_VOID
}
void GenerateConsolidatedRotationKeys(int* galEls, int n) {
  API_BEGIN
  Context& c = ctx();
  for (int i = 0; i < n; ++i) {
    const u64 g = (u64)(unsigned)galEls[i];
    if (g != 1) c.gen_galois(g, c.hinted_level(g));
  }
  API_END_VOID
}
// lineartransform.go:131-142: a fresh key, serialised and NOT kept (the
// save path stores it to HDF5 and LoadRotationKey brings it back per layer).
// Like Lattigo's GenGaloisKeyNew the blob is a full-chain key (every digit over
// every Q limb); LoadRotationKey scopes it to the level its transforms need.
ArrayResultByte GenerateAndSerializeRotationKey(int galEl) {
  ArrayResultByte r{nullptr, 0};
  API_BEGIN
  Context& c = ctx();
  const u64 g = (u64)(unsigned)galEl;
  auto kept = c.gks.find(g);
  EvKey saved;
  if (kept != c.gks.end()) {
    saved = kept->second;
    c.gks.erase(kept);
  }
  const int level = c.L - 1;
  c.gen_galois(g, level);
  std::vector<u64> host;
  c.download(c.gks.at(g).k, host);
  c.gks.erase(g);
  if (saved.k.buf) c.gks[g] = saved;
  return to_bytes(galois_key_bytes(c, g, host, level));
  API_END(r)
}
// lineartransform.go:145-164: unmarshal an rlwe.GaloisKey into the key set under
// galEl.  A key asked for by a linear transform is kept only over the limbs and
// digits of the highest level that uses it (key_hint): the digits 0..beta-1 of
// a key made for a higher level, restricted to q_0..q_level and P, are exactly
// the key Lattigo's gadget product reads at that level.
void LoadRotationKey(char* data, unsigned long len, unsigned long galEl) {
  API_BEGIN
  Context& c = ctx();
  if (!data) throw std::runtime_error("null rotation key data");
  wire::Reader rd(data, len);
  const u64 ge = rd.get_u64(), nth = rd.get_u64(), b2 = rd.get_u64(), rows = rd.get_u64();
  if (nth != c.nthroot) throw std::runtime_error("rotation key: NthRoot does not match the ring");
  if (b2 != 0) throw std::runtime_error("rotation key: power-of-two decomposition is not supported");
  if (ge != galEl) throw std::runtime_error("rotation key: blob is for Galois element " + std::to_string(ge));
  if (rows < 1 || rows > (u64)c.dnum) throw std::runtime_error("rotation key: gadget rows outside 1..dnum");
  if (rd.get_u64() != 1 || rd.get_u64() != 2) throw std::runtime_error("rotation key: unexpected gadget shape");
  // the level the key was made for: its Q limb count (peeked from the first ring.Poly)
  const u64 nq = rd.get_u64();
  if (nq < 1 || nq > (u64)c.L) throw std::runtime_error("rotation key: Q limb count outside the chain");
  const int level = (int)nq - 1, beta = (level + 1 + c.K - 1) / c.K;
  if (rows != (u64)beta) throw std::runtime_error("rotation key: gadget rows do not match its level");
  wire::Reader body(data + 48, len - 48);  // past the 4-word header and row 0's column/vector lengths
  const size_t qp = (size_t)(level + 1 + c.K) * c.N;
  std::vector<u64> host(2 * (size_t)beta * qp);
  for (int i = 0; i < beta; ++i) {
    if (i && (body.get_u64() != 1 || body.get_u64() != 2))
      throw std::runtime_error("rotation key: unexpected gadget shape");
    for (int k = 0; k < 2; ++k) get_qp(body, c, host.data() + (2 * (size_t)i + k) * qp, level + 1, "rotation key");
  }
  if (body.left()) throw std::runtime_error("rotation key blob has trailing bytes");
  const int tl = std::min(level, c.hinted_level(galEl)), tbeta = (tl + 1 + c.K - 1) / c.K;
  if (tl < level) {  // keep digits < tbeta over limbs q_0..q_tl, p_0..p_{K-1}
    const size_t tqp = (size_t)(tl + 1 + c.K) * c.N;
    std::vector<u64> sc(2 * (size_t)tbeta * tqp);
    for (int r = 0; r < 2 * tbeta; ++r) {
      const u64* src = host.data() + (size_t)r * qp;
      u64* dst = sc.data() + (size_t)r * tqp;
      memcpy(dst, src, sizeof(u64) * (size_t)(tl + 1) * c.N);
      memcpy(dst + (size_t)(tl + 1) * c.N, src + (size_t)(level + 1) * c.N, sizeof(u64) * (size_t)c.K * c.N);
    }
    // the whole key stays in host memory (as Lattigo keeps it,
    // lineartransform.go:143-159): a later use above tl uploads it whole
    c.gk_host[galEl] = Context::HostKey{level, std::make_shared<const std::vector<u64>>(std::move(host))};
    host = std::move(sc);
  } else {
    c.gk_host.erase(galEl);
  }
  Poly k = c.alloc(2 * tbeta, tl + 1 + c.K, 1);
  c.upload(k, host);
  c.gks[galEl] = EvKey{k, tl};
  API_END_VOID
}
// lineartransform.go:167-183: the diagonal's ringqp.Poly (Q at the transform's
// level, P), after which the transform forgets it until LoadPlaintextDiagonal
ArrayResultByte SerializeDiagonal(int tid, int diagIdx) {
  ArrayResultByte r{nullptr, 0};
  API_BEGIN
  Context& c = ctx();
  LinTrans& T = c.lts.get(tid);
  const int key = diagIdx & (c.slots - 1);
  auto it = T.diags.find(key);
  if (it == T.diags.end()) throw std::runtime_error("diagonal " + std::to_string(diagIdx) + " is not loaded");
  std::vector<u64> host;
  c.download(it->second.poly, host);
  std::vector<char> bytes;
  put_qp(bytes, c, host.data(), T.level + 1);
  T.diags.erase(it);
  T.sdiags.erase(key);
  T.plan_dirty = true;
  c.lts.touch(tid);  // (a pipeline reading it waits for this context's work again)
  return to_bytes(bytes);
  API_END(r)
}
// lineartransform.go:186-200
void LoadPlaintextDiagonal(char* data, unsigned long len, int tid, unsigned long diagIdx) {
  API_BEGIN
  Context& c = ctx();
  if (!data) throw std::runtime_error("null diagonal data");
  LinTrans& T = c.lts.get(tid);
  Plaintext p;
  p.level = T.level;
  p.qp = true;
  p.scale = (long double)c.mods[T.level];
  p.poly = c.alloc(1, T.level + 1 + c.K, 1);
  wire::Reader rd(data, len);
  std::vector<u64> host((size_t)p.poly.nlimb * c.N);
  get_qp(rd, c, host.data(), T.level + 1, "diagonal");
  if (rd.left()) throw std::runtime_error("diagonal blob has trailing bytes");
  c.upload(p.poly, host);
  T.diags[(int)diagIdx & (c.slots - 1)] = p;
  T.plan_dirty = true;
  c.lts.touch(tid);
  API_END_VOID
}
void RemovePlaintextDiagonals(int tid) {
  API_BEGIN
  ctx().lts.get(tid).diags.clear();
  ctx().lts.get(tid).sdiags.clear();
  ctx().lts.get(tid).plan_dirty = true;
  ctx().lts.touch(tid);
  API_END_VOID
}
void RemoveRotationKeys(void) {
  API_BEGIN
  ctx().gks.clear();
  ctx().gk_host.clear();
  API_END_VOID
}

// ---- SURVEY §8f "next": polynomial evaluation, minimax, bootstrapping ----
void NewPolynomialEvaluator(void) {}
static int add_poly(float* coeffs, int n, bool cheb) {
  Context& c = ctx();
  if (!coeffs || n < 1) throw std::runtime_error("polynomial needs at least one coefficient");
  Context::PolyFn p;
  p.cheb = cheb;
  for (int i = 0; i < n; ++i) p.c.push_back((long double)coeffs[i]);
  return c.polys.add(std::move(p));
}
// polyeval.go:38-47: bignum.Monomial, coefficients lowest degree first
int GenerateMonomial(float* coeffs, int n) {
  API_BEGIN
  return add_poly(coeffs, n, false);
  API_END(-1)
}
// polyeval.go:50-60: bignum.Chebyshev on [-1, 1]
int GenerateChebyshev(float* coeffs, int n) {
  API_BEGIN
  return add_poly(coeffs, n, true);
  API_END(-1)
}
// poly_evaluator.py:58-59: levels an evaluation consumes, bits.Len64(degree)
int GetPolyDepth(int poly) {
  API_BEGIN
  const int deg = (int)ctx().polys.get(poly).c.size() - 1;
  int d = 0;
  while ((1 << d) <= deg) ++d;
  return d;
  API_END(-1)
}
// polyeval.go:63-84: a new ciphertext at level - bitlen(degree), scale outScale
int EvaluatePolynomial(int ct, int poly, unsigned long outScale) {
  API_BEGIN
  Context& c = ctx();
  return c.cts.add(c.eval_poly(c.cts.get(ct), c.polys.get(poly), (long double)outScale));
  API_END(-1)
}
// polyeval.go:91-167: composite minimax sign coefficients (compile-time, host),
// cached per (degrees, prec, logalpha, logerr) like minimaxSignMap; every fit
// absorbs the scheme error 2^-logerr, and the last polynomial is mapped from
// [-1, 1] to [0, 1] (halved, + 0.5, inside minimax_sign_composite).  The Remez
// restatement works in binary128 / double-binary128 whatever `prec` asks for:
// at prec >= 113 (orion's default is 128) the doubles are the prec-bit
// computation's (tests/golden/minimax_sign.json).
static std::map<std::string, std::vector<double>> g_minimax_cache;
ArrayResultDouble GenerateMinimaxSignCoeffs(int* degrees, int n, int prec, int logalpha, int logerr, int debug) {
  ArrayResultDouble r{nullptr, 0};
  API_BEGIN
  std::vector<int> deg;
  for (int i = 0; i < n; ++i) deg.push_back(degrees[i]);
  if (deg.empty()) throw std::runtime_error("at least one degree is required");
  std::string key;
  for (int d : deg) key += std::to_string(d) + ",";
  key += "|" + std::to_string(prec) + "|" + std::to_string(logalpha) + "|" + std::to_string(logerr);
  auto it = g_minimax_cache.find(key);
  if (it == g_minimax_cache.end()) {
    std::vector<std::vector<double>> polys = minimax_sign_composite(deg, logalpha, logerr, nullptr, debug != 0);
    std::vector<double> flat;
    for (auto& p : polys) flat.insert(flat.end(), p.begin(), p.end());
    it = g_minimax_cache.emplace(key, flat).first;
  }
  r.Data = to_c_array<double, double>(it->second, &r.Length);
  return r;
  API_END(r)
}
// bootstrapper.go:19-58: one bootstrapper per slot count, made once, under
// bootstrapping parameters with P primes of the bit sizes logPs
// (Context::new_bootstrapper)
void NewBootstrapper(int* logPs, int n, int slots) {
  API_BEGIN
  Context& c = ctx();
  std::vector<int> lp;
  if (logPs && n > 0) lp.assign(logPs, logPs + n);
  c.new_bootstrapper(lp, slots);
  API_END_VOID
}
// bootstrapper.go:61-80: a new ciphertext refreshed to the residual top level,
// at the input's scale, post-scaled by 2^(LogMaxSlots - LogSlots)
int Bootstrap(int ct, int slots) {
  API_BEGIN
  Context& c = ctx();
  Context* s = scheme_ctx();
  if (c.btps.count(slots) || !s || s == &c) return c.cts.add(c.bootstrap(c.cts.get(ct), slots));
  // a pipeline bootstraps with the scheme's bootstrapper (one circuit and key
  // set per process), on the scheme's stream under the scheme's lock: the
  // scheme's stream waits for the input, the result is copied into a buffer
  // of this pipeline's pool there, and this stream waits for the copy
  const Ciphertext& in = c.cts.get(ct);
  std::lock_guard<std::recursive_mutex> lk(s->mu);  // (a pipeline may wait on the scheme: index order)
  wait_on(*s, c);
  Ciphertext out;
  {
    Context* saved = t_act;
    t_act = s;
    try {
      Ciphertext r = s->bootstrap(in, slots);
      out = c.new_ct(r.level, r.poly.B, r.scale);
      s->copy(s->lsq(out.poly, 0, 2, r.level), s->lsq(r.poly, 0, 2, r.level));
    } catch (...) {
      t_act = saved;
      throw;
    }
    t_act = saved;
  }
  wait_on(c, *s);
  return c.cts.add(std::move(out));
  API_END(-1)
}
void DeleteBootstrappers(void) {
  API_BEGIN
  if (t_act) t_act->delete_bootstrappers();
  API_END_VOID
}
// the bootstrapping chain of the circuit for `slots` (its Q primes, then its P primes)
static Context* btp_context(int slots) {
  Context* s = scheme_ctx();
  if (!s) return nullptr;
  auto it = s->btps.find(slots);
  return it == s->btps.end() ? nullptr : it->second->bc;
}
int OrionHipBootstrapNumQ(int slots) {
  Context* b = btp_context(slots);
  return b ? b->L : -1;
}
int OrionHipBootstrapNumP(int slots) {
  Context* b = btp_context(slots);
  return b ? b->K : -1;
}
unsigned long OrionHipBootstrapModulus(int slots, int i) {
  Context* b = btp_context(slots);
  return (b && i >= 0 && i < (int)b->mods.size()) ? b->mods[i] : 0;
}

// an evaluation key in the full-chain layout [dnum][2][L+K][N]: a key made for
// a lower level fills its digits and limbs, the rest is zero
static void export_evk_full(Context& c, const EvKey& k, unsigned long* out, unsigned long n) {
  if (n != (unsigned long)2 * c.dnum * (c.L + c.K) * c.N) throw std::runtime_error("export buffer size mismatch");
  std::vector<u64> host;
  c.download(k.k, host);
  memset(out, 0, n * 8);
  const int beta = k.k.ncomp / 2, nl = k.k.nlimb;
  for (int i = 0; i < 2 * beta; ++i)
    for (int x = 0; x < nl; ++x) {
      const int m = x <= k.level ? x : c.L + (x - k.level - 1);
      memcpy(out + ((size_t)i * (c.L + c.K) + m) * c.N, host.data() + ((size_t)i * nl + x) * c.N, (size_t)c.N * 8);
    }
}

// Parity access to a bootstrapper's shared inputs (tests/test_gpu_parity.py
// bootstrapping parity; the CPU oracle restates the circuit from them):
// returns the element count written (or needed, out = NULL), -1 on error.
long OrionHipBootstrapExport(int slots, int what, long arg, void* out, unsigned long n) {
  API_BEGIN
  Context& c = ctx();
  auto it = c.btps.find(slots);
  if (it == c.btps.end()) throw std::runtime_error("no bootstrapper found for slot count: " + std::to_string(slots));
  Context::Bootstrapper& bt = *it->second;
  Context& b = *bt.bc;
  auto lt_of = [&](long i) -> LinTrans& {
    if (i < 0 || i >= (long)(bt.cts.size() + bt.stc.size())) throw std::runtime_error("bootstrap LT index out of range");
    return i < (long)bt.cts.size() ? bt.cts[i] : bt.stc[i - bt.cts.size()];
  };
  switch (what) {
    case ORION_BTX_PARAMS: {  // long double: F, gap, K, r, degree, slots, s_y, top, L, K_P, ntrace, nlt, degree+1, t0
      const long double v[] = {(long double)bt.F, (long double)bt.gap, (long double)bt.K, (long double)bt.r,
                               (long double)bt.degree, (long double)bt.slots, bt.s_y, (long double)bt.top,
                               (long double)b.L, (long double)b.K, (long double)bt.trace_gal.size(),
                               (long double)(bt.cts.size() + bt.stc.size()), (long double)bt.cosp.c.size(), bt.t0};
      const long cnt = (long)(sizeof(v) / sizeof(v[0]));
      if (out) {
        if (n < (unsigned long)cnt) throw std::runtime_error("export buffer too small");
        memcpy(out, v, sizeof(v));
      }
      return cnt;
    }
    case ORION_BTX_COS: {
      const long cnt = (long)bt.cosp.c.size();
      if (out) {
        if (n < (unsigned long)cnt) throw std::runtime_error("export buffer too small");
        for (long i = 0; i < cnt; ++i) ((long double*)out)[i] = bt.cosp.c[i];
      }
      return cnt;
    }
    case ORION_BTX_TRACE: {
      const long cnt = (long)bt.trace_gal.size();
      if (out) {
        if (n < (unsigned long)cnt) throw std::runtime_error("export buffer too small");
        for (long i = 0; i < cnt; ++i) ((unsigned long*)out)[i] = bt.trace_gal[i];
      }
      return cnt;
    }
    case ORION_BTX_RLK: {
      const long cnt = 2L * b.dnum * (b.L + b.K) * b.N;
      if (out) export_evk_full(b, EvKey{b.rlk, b.L - 1}, (unsigned long*)out, n);
      return cnt;
    }
    case ORION_BTX_GALOIS_KEYS: {  // the Galois elements with a key in the bootstrapping context
      const long cnt = (long)b.gks.size();
      if (out) {
        if (n < (unsigned long)cnt) throw std::runtime_error("export buffer too small");
        long i = 0;
        for (auto& kv : b.gks) ((unsigned long*)out)[i++] = kv.first;
      }
      return cnt;
    }
    case ORION_BTX_GALOIS: {
      auto kt = b.gks.find((u64)arg);
      if (kt == b.gks.end()) throw std::runtime_error("no galois key for element " + std::to_string(arg));
      const long cnt = 2L * b.dnum * (b.L + b.K) * b.N;
      if (out) export_evk_full(b, kt->second, (unsigned long*)out, n);
      return cnt;
    }
    case ORION_BTX_LT_INFO: {  // long: level, N1, ndiag, then the diagonal indices
      LinTrans& T = lt_of(arg);
      const long cnt = 3 + (long)T.idx.size();
      if (out) {
        if (n < (unsigned long)cnt) throw std::runtime_error("export buffer too small");
        long* o = (long*)out;
        o[0] = T.level, o[1] = T.N1, o[2] = (long)T.idx.size();
        for (size_t k = 0; k < T.idx.size(); ++k) o[3 + k] = T.idx[k];
      }
      return cnt;
    }
    case ORION_BTX_LT_DIAG: {  // arg = lt * 2^32 + k: the k-th diagonal (QP plaintext [level+1+K][N])
      LinTrans& T = lt_of(arg >> 32);
      const long k = arg & 0xffffffffl;
      if (k < 0 || k >= (long)T.idx.size()) throw std::runtime_error("bootstrap LT diagonal index out of range");
      const Poly& p = T.diags.at(T.idx[k] & (b.N / 2 - 1)).poly;
      const long cnt = (long)p.nlimb * b.N;
      if (out) {
        if (n != (unsigned long)cnt) throw std::runtime_error("export buffer size mismatch");
        std::vector<u64> host;
        b.download(p, host);
        memcpy(out, host.data(), (size_t)cnt * 8);
      }
      return cnt;
    }
    case ORION_BTX_D2S:  // the ephemeral-secret keys (full-chain layout; EvkDenseToSparse fills level 0)
    case ORION_BTX_S2D: {
      const long cnt = 2L * b.dnum * (b.L + b.K) * b.N;
      if (out) export_evk_full(b, what == ORION_BTX_D2S ? bt.d2s : bt.s2d, (unsigned long*)out, n);
      return cnt;
    }
    case ORION_BTX_MONO_I: {
      if (!bt.mono_i.buf) throw std::runtime_error("sparse-slot circuit: no X^(N/2) plaintext");
      const long cnt = (long)bt.mono_i.nlimb * b.N;
      if (out) {
        if (n != (unsigned long)cnt) throw std::runtime_error("export buffer size mismatch");
        std::vector<u64> host;
        b.download(bt.mono_i, host);
        memcpy(out, host.data(), (size_t)cnt * 8);
      }
      return cnt;
    }
    default:
      throw std::runtime_error("unknown bootstrap export item " + std::to_string(what));
  }
  API_END(-1)
}

// ---- import / export ----
static void to_canonical(const std::vector<u64>& dev, int ncomp, int nl, int B, int N, unsigned long* out) {
  // device [c][l][b][n] -> host [b][c][l][n]
  for (int c = 0; c < ncomp; ++c)
    for (int l = 0; l < nl; ++l)
      for (int b = 0; b < B; ++b)
        memcpy(out + (((size_t)b * ncomp + c) * nl + l) * N, dev.data() + (((size_t)c * nl + l) * B + b) * N, N * 8);
}
static std::vector<u64> from_canonical(const unsigned long* in, int ncomp, int nl, int B, int N) {
  std::vector<u64> dev((size_t)ncomp * nl * B * N);
  for (int c = 0; c < ncomp; ++c)
    for (int l = 0; l < nl; ++l)
      for (int b = 0; b < B; ++b)
        memcpy(dev.data() + (((size_t)c * nl + l) * B + b) * N, in + (((size_t)b * ncomp + c) * nl + l) * N, N * 8);
  return dev;
}
static void check_import(const Context& c, const void* data, int B, int level) {
  if (!data) throw std::runtime_error("null data pointer");
  if (level < 0 || level >= c.L || B < 1) throw std::runtime_error("invalid level/batch");
}
int ImportCiphertext(const unsigned long* data, int B, int level, double scale) {
  API_BEGIN
  Context& c = ctx();
  check_import(c, data, B, level);
  Ciphertext ct = c.new_ct(level, B, (long double)scale);
  c.upload(ct.poly, from_canonical(data, 2, level + 1, B, c.N));
  return c.cts.add(std::move(ct));
  API_END(-1)
}
int ExportCiphertext(int id, unsigned long* out, unsigned long n) {
  API_BEGIN
  Context& c = ctx();
  const Ciphertext& ct = c.cts.get(id);
  const int nl = ct.level + 1, B = ct.poly.B;
  if (n != (unsigned long)B * 2 * nl * c.N) throw std::runtime_error("export buffer size mismatch");
  Poly t = c.alloc(2, nl, B);
  c.copy(c.lsq(t, 0, 2, ct.level), c.lsq(ct.poly, 0, 2, ct.level));
  std::vector<u64> host;
  c.download(t, host);
  to_canonical(host, 2, nl, B, c.N, out);
  return 0;
  API_END(-1)
}
// canonical [B][2][nl][N] device layout <-> the library's [2][nl][B][N]: one
// strided 2-D copy per (comp, limb) plane, no host round trip
static void copy_planes(Context& c, u64* dst, long long dpitch, const u64* src, long long spitch, int nplane, int B,
                        long long dplane, long long splane) {
  for (int p = 0; p < nplane; ++p)
    HIPCHK(hipMemcpy2DAsync(dst + p * dplane, dpitch * 8, src + p * splane, spitch * 8, (size_t)c.N * 8, B,
                            hipMemcpyDeviceToDevice, c.stream));
}
int ImportCiphertextDevice(const unsigned long* dptr, int B, int level, double scale) {
  API_BEGIN
  Context& c = ctx();
  check_import(c, dptr, B, level);
  const int nl = level + 1;
  Ciphertext ct = c.new_ct(level, B, (long double)scale);
  // plane (comp, limb) = p: library offset p*B*N, canonical offset p*N with row pitch 2*nl*N
  copy_planes(c, ct.poly.ptr(), c.N, (const u64*)dptr, (long long)2 * nl * c.N, 2 * nl, B, (long long)B * c.N, c.N);
  return c.cts.add(std::move(ct));
  API_END(-1)
}
int ExportCiphertextDevice(int id, unsigned long* dptr, unsigned long n) {
  API_BEGIN
  Context& c = ctx();
  if (!dptr) throw std::runtime_error("null output pointer");
  const Ciphertext& ct = c.cts.get(id);
  const int nl = ct.level + 1, B = ct.poly.B;
  if (n != (unsigned long)B * 2 * nl * c.N) throw std::runtime_error("export buffer size mismatch");
  // a ciphertext's limb planes may be allocated for a higher level: address them by its strides
  const Poly& P = ct.poly;
  for (int comp = 0; comp < 2; ++comp)
    for (int l = 0; l < nl; ++l)
      HIPCHK(hipMemcpy2DAsync((u64*)dptr + ((size_t)comp * nl + l) * c.N, (size_t)2 * nl * c.N * 8,
                              P.ptr() + comp * P.comp_stride() + l * P.limb_stride(), (size_t)c.N * 8,
                              (size_t)c.N * 8, B, hipMemcpyDeviceToDevice, c.stream));
  return 0;
  API_END(-1)
}
int ImportPlaintext(const unsigned long* data, int B, int level, double scale) {
  API_BEGIN
  Context& c = ctx();
  check_import(c, data, B, level);
  Plaintext p;
  p.level = level;
  p.scale = (long double)scale;
  p.poly = c.alloc(1, level + 1, B);
  c.upload(p.poly, from_canonical(data, 1, level + 1, B, c.N));
  return c.pts.add(std::move(p));
  API_END(-1)
}
int ExportPlaintext(int id, unsigned long* out, unsigned long n) {
  API_BEGIN
  Context& c = ctx();
  const Plaintext& p = c.pts.get(id);
  const int nl = p.poly.nlimb, B = p.poly.B;
  if (n != (unsigned long)B * nl * c.N) throw std::runtime_error("export buffer size mismatch");
  std::vector<u64> host;
  c.download(p.poly, host);
  to_canonical(host, 1, nl, B, c.N, out);
  return 0;
  API_END(-1)
}
static int export_poly(const Poly& p, unsigned long* out, unsigned long n) {
  Context& c = ctx();
  std::vector<u64> host;
  c.download(p, host);
  if (n != host.size()) throw std::runtime_error("export buffer size mismatch");
  memcpy(out, host.data(), n * 8);
  return 0;
}
int ExportSecretKey(unsigned long* out, unsigned long n) {
  API_BEGIN
  if (!ctx().have_sk) throw std::runtime_error("no secret key");
  return export_poly(ctx().sk, out, n);
  API_END(-1)
}
int ExportPublicKey(unsigned long* out, unsigned long n) {
  API_BEGIN
  if (!ctx().have_pk) throw std::runtime_error("no public key");
  return export_poly(ctx().pk, out, n);
  API_END(-1)
}
unsigned int OrionHipEncryptionIndex(void) {
  API_BEGIN
  return t_act ? t_act->enc_sampler.enc : 0;
  API_END(0)
}
int ExportRelinKey(unsigned long* out, unsigned long n) {
  API_BEGIN
  if (!ctx().have_rlk) throw std::runtime_error("no relinearization key");
  return export_poly(ctx().rlk, out, n);
  API_END(-1)
}
int ExportGaloisKey(unsigned long galEl, unsigned long* out, unsigned long n) {
  API_BEGIN
  Context& c = ctx();
  auto it = c.gks.find(galEl);
  if (it == c.gks.end()) throw std::runtime_error("no galois key for element " + std::to_string(galEl));
  export_evk_full(c, it->second, out, n);  // the full-chain layout [dnum][2][L+K][N]
  return 0;
  API_END(-1)
}
int GetGaloisKeyLevel(unsigned long galEl) {
  API_BEGIN
  Context& c = ctx();
  auto it = c.gks.find(galEl);
  if (it == c.gks.end()) throw std::runtime_error("no galois key for element " + std::to_string(galEl));
  return it->second.level;
  API_END(-1)
}
int ExportLinearTransformDiagonal(int tid, int diagIdx, unsigned long* out, unsigned long n) {
  API_BEGIN
  Context& c = ctx();
  return export_poly(c.lts.get(tid).diags.at(diagIdx & (c.slots - 1)).poly, out, n);
  API_END(-1)
}

// ---- key bundle for RCCL broadcast ----
// layout: header u64[KB_HDR] {magic, ngk, withSecret, haveRlk, logN, L, K,
// dnum, moduli digest}, galEls[ngk], then pk, rlk, gk_0..gk_{ngk-1}, [sk] as
// raw device polys.  The importer rejects a bundle made for another chain.
enum { KB_HDR = 9 };
static const u64 KB_MAGIC = 0x4f52494f4e4b4232ull;  // "ORIONKB2"
static u64 moduli_digest(const Context& c) {
  u64 h = 0xcbf29ce484222325ull;  // FNV-1a over the QP moduli
  for (u64 q : c.mods)
    for (int b = 0; b < 8; ++b) h = (h ^ ((q >> (8 * b)) & 0xff)) * 0x100000001b3ull;
  return h;
}
unsigned long KeyBundleBytes(int withSecret) {
  API_BEGIN
  Context& c = ctx();
  const size_t key = (size_t)2 * c.dnum * (c.L + c.K) * c.N * 8, pk = (size_t)2 * (c.L + c.K) * c.N * 8,
               sk = (size_t)(c.L + c.K) * c.N * 8;
  size_t hdr = (KB_HDR + 2 * c.gks.size()) * 8;
  hdr = (hdr + 255) & ~(size_t)255;
  size_t gk = 0;
  for (auto& kv : c.gks) gk += (size_t)kv.second.k.ncomp * kv.second.k.nlimb * c.N * 8;
  return hdr + pk + (c.have_rlk ? key : 0) + gk + (withSecret ? sk : 0);
  API_END(0)
}
int ExportKeyBundle(void* dptr, int withSecret) {
  API_BEGIN
  Context& c = ctx();
  if (!dptr) throw std::runtime_error("null bundle pointer");
  if (!c.have_pk) throw std::runtime_error("no public key");
  if (withSecret && !c.have_sk) throw std::runtime_error("no secret key");
  std::vector<u64> hdr = {KB_MAGIC, (u64)c.gks.size(), (u64)(withSecret ? 1 : 0), (u64)c.have_rlk,
                          (u64)c.logN, (u64)c.L, (u64)c.K, (u64)c.dnum, moduli_digest(c)};
  for (auto& kv : c.gks) hdr.push_back(kv.first), hdr.push_back((u64)kv.second.level);
  size_t off = ((hdr.size() * 8) + 255) & ~(size_t)255;
  char* d = (char*)dptr;
  HIPCHK(hipMemcpyAsync(d, hdr.data(), hdr.size() * 8, hipMemcpyHostToDevice, c.stream));
  auto put = [&](const Poly& p) {
    const size_t b = (size_t)p.ncomp * p.nlimb * p.B * c.N * 8;
    HIPCHK(hipMemcpyAsync(d + off, p.ptr(), b, hipMemcpyDeviceToDevice, c.stream));
    off += b;
  };
  put(c.pk);
  if (c.have_rlk) put(c.rlk);
  for (auto& kv : c.gks) put(kv.second.k);
  if (withSecret) put(c.sk);
  HIPCHK(hipStreamSynchronize(c.stream));
  return 0;
  API_END(-1)
}
int ImportKeyBundle(const void* dptr, unsigned long bytes) {
  API_BEGIN
  Context& c = ctx();
  if (!dptr) throw std::runtime_error("null bundle pointer");
  if (bytes < KB_HDR * 8) throw std::runtime_error("key bundle shorter than its header");
  u64 h4[KB_HDR];
  HIPCHK(hipMemcpy(h4, dptr, sizeof(h4), hipMemcpyDeviceToHost));
  if (h4[0] != KB_MAGIC) throw std::runtime_error("not a key bundle");
  if (h4[4] != (u64)c.logN || h4[5] != (u64)c.L || h4[6] != (u64)c.K || h4[7] != (u64)c.dnum ||
      h4[8] != moduli_digest(c))
    throw std::runtime_error("key bundle was made for another modulus chain (logN/L/K/dnum/moduli differ)");
  if (h4[1] > (bytes / 8 - KB_HDR) / 2) throw std::runtime_error("key bundle truncated (galois element list)");
  std::vector<u64> gels(2 * h4[1]);  // (element, level) pairs
  if (h4[1]) HIPCHK(hipMemcpy(gels.data(), (const char*)dptr + KB_HDR * 8, h4[1] * 16, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < h4[1]; ++i)
    if (gels[2 * i + 1] >= (u64)c.L) throw std::runtime_error("key bundle: galois key level outside the chain");
  size_t off = ((KB_HDR + 2 * h4[1]) * 8 + 255) & ~(size_t)255;
  const char* d = (const char*)dptr;
  auto get = [&](int ncomp, int nlimb) {
    Poly p = c.alloc(ncomp, nlimb, 1);
    const size_t b = (size_t)ncomp * nlimb * c.N * 8;
    if (off + b > bytes) throw std::runtime_error("key bundle truncated");
    HIPCHK(hipMemcpyAsync(p.ptr(), d + off, b, hipMemcpyDeviceToDevice, c.stream));
    off += b;
    return p;
  };
  c.pk = get(2, c.L + c.K);
  c.have_pk = true;
  if (h4[3]) {
    c.rlk = get(2 * c.dnum, c.L + c.K);
    c.have_rlk = true;
  }
  for (size_t i = 0; i < h4[1]; ++i) {
    const int lv = (int)gels[2 * i + 1];
    c.gks[gels[2 * i]] = EvKey{get(2 * ((lv + 1 + c.K - 1) / c.K), lv + 1 + c.K), lv};
  }
  if (h4[2]) {
    c.sk = get(1, c.L + c.K);
    c.have_sk = true;
  }
  HIPCHK(hipStreamSynchronize(c.stream));
  return 0;
  API_END(-1)
}

// ---- profiling ----
// Profiling switches and counters cover every context of the scheme (the
// pipelines' launches included); each context is locked on its own in turn.
}  // extern "C"
template <class F>
static void each_ctx(F f) {
  for (int i = 0; i < g_nctx.load(); ++i) {
    Context* c = g_slot[i].get();
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    f(*c);
    // the bootstrapping contexts the context owns (their launches run under its lock)
    for (auto& kv : c->btp_ctx) f(*kv.second);
  }
}
extern "C" {
void OrionHipProfile(int enable) {
  API_BEGIN_NOCTX
  each_ctx([&](Context& c) {
    if (!enable) c.prof_flush();
    c.prof = enable == 1 ? 0xffffffffu : (unsigned)enable;  // 1 = all categories, else a bit mask
  });
  API_END_VOID
}
// the reference of the union timing: recorded on the scheme's stream once
// every context is drained; the intervals collected so far are dropped
void OrionHipProfileClock(void) {
  API_BEGIN_NOCTX
  Context* s = scheme_ctx();
  if (!s) throw std::runtime_error("scheme not initialised: call NewScheme first");
  each_ctx([](Context& c) { c.prof_flush(); });
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_iv.clear();
  if (!g_prof_ref) HIPCHK(hipEventCreate(&g_prof_ref));
  HIPCHK(hipEventRecord(g_prof_ref, s->stream));
  HIPCHK(hipEventSynchronize(g_prof_ref));
  API_END_VOID
}
// the union of the wall-clock intervals of every context's profiled launches
// of the categories in `mask` since OrionHipProfileClock (ms): e.g. the time
// at least one NTT ran while pipelines overlap
double OrionHipProfileUnion(unsigned mask) {
  API_BEGIN_NOCTX
  each_ctx([](Context& c) { c.prof_flush(); });
  std::vector<std::pair<float, float>> iv;
  {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (const ProfIv& r : g_prof_iv)
      if (mask & (1u << r.cat)) iv.push_back({r.t0, r.t1});
  }
  std::sort(iv.begin(), iv.end());
  double tot = 0;
  float b = 0, e = 0;
  bool open = false;
  for (auto& x : iv) {
    if (!open || x.first > e) {
      if (open) tot += e - b;
      b = x.first, e = x.second, open = true;
    } else if (x.second > e) {
      e = x.second;
    }
  }
  if (open) tot += e - b;
  return tot;
  API_END(-1.0)
}
// a marker line ("# tag") in the NTT call log (bench.py brackets its timed
// region, so a kernel trace can be cut to it)
void OrionHipLogMark(const char* tag) {
  if (FILE* f = ntt_log_file()) fprintf(f, "# %s\n", tag ? tag : "");
}
void OrionHipProfileReset(void) {
  API_BEGIN_NOCTX
  each_ctx([](Context& c) {
    c.prof_flush();
    for (int i = 0; i < P_NCAT; ++i) c.prof_launch[i] = c.prof_ms[i] = c.prof_bytes[i] = c.prof_strict[i] = 0;
  });
  API_END_VOID
}
// counters summed over every context
int OrionHipProfileRead(char* names, long* launches, double* ms, double* bytes, int max) {
  API_BEGIN_NOCTX
  int n = std::min(max, (int)P_NCAT);
  for (int i = 0; i < n; ++i) {
    strncpy(names + 32 * i, kProfNames[i], 31);
    names[32 * i + 31] = 0;
    launches[i] = 0;
    ms[i] = bytes[i] = 0;
  }
  each_ctx([&](Context& c) {
    c.prof_flush();
    for (int i = 0; i < n; ++i) {
      launches[i] += (long)c.prof_launch[i];
      ms[i] += c.prof_ms[i];
      bytes[i] += c.prof_bytes[i];
    }
  });
  return n;
  API_END(-1)
}
int OrionHipProfileReadStrict(double* strict, int max) {
  API_BEGIN_NOCTX
  int n = std::min(max, (int)P_NCAT);
  for (int i = 0; i < n; ++i) strict[i] = 0;
  each_ctx([&](Context& c) {
    c.prof_flush();
    for (int i = 0; i < n; ++i) strict[i] += c.prof_strict[i];
  });
  return n;
  API_END(-1)
}

int OrionHipNTT(unsigned long* dptr, int nlimb, int batch, const int* mods, int inverse) {
  API_BEGIN
  Context& c = ctx();
  LimbSet s;
  memset(&s, 0, sizeof(s));
  s.p = (u64*)dptr;
  s.ncomp = 1;
  s.nlimb = nlimb;
  s.nbatch = batch;
  s.batch_stride = c.N;
  s.limb_stride = (long long)batch * c.N;
  if (nlimb > ORION_MAXLIMB) throw std::runtime_error("too many limbs");
  for (int l = 0; l < nlimb; ++l) {
    if (mods[l] < 0 || mods[l] >= c.L + c.K) throw std::runtime_error("bad modulus index");
    s.mod[l] = (unsigned char)mods[l];
    s.pos[l] = (unsigned char)l;
  }
  c.ntt(s, inverse != 0);
  return 0;
  API_END(-1)
}

}  // extern "C"
