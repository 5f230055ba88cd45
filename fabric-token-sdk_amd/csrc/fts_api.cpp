// C-ABI of the MI355X zkatdlog batch verifier (include/fts_gpu.h).
//
// Host side of the drop-in boundary: context creation from the public
// parameters (setup.go:319-372), DER decoding of proofs into device records,
// orchestration of the HIP kernels in rp_kernels.hip / sigma_kernels.hip, and
// the reference error-precedence rules (transfer.go:153-197,
// issue/verifier.go:32-57, rangecorrectness.go:137-162).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <sys/random.h>
#include <vector>

#include "../../include/fts_gpu.h"
#include "device/rp_kernels.hpp"
#include "device/sigma.hpp"
#include "device/prove.hpp"
#include "host/bn254_host.hpp"
#include "host/der.hpp"
#include "host/pp_parse.hpp"
#include "host/request_parse.hpp"
#include "host/proofs.hpp"
#include "host/prover.hpp"
#include "device/wave_prio.hpp"

namespace fts {
// device launchers (rp_kernels.hip)

size_t rp_scratch_words(int B, int n, int k);
size_t rp_terms_words(int B, int n, int k);
void launch_build_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s);
void launch_rp_batch(const RpBatchDev& d, const RlcDev& r, const uint32_t* tables, const uint32_t* wtables,
                     const uint8_t* x0_const, const uint8_t* x0_tmpl, hipStream_t s, hipStream_t s2, hipStream_t s3,
                     hipStream_t s4,
                     Timeline* tl, int wbits);
void launch_build_wide_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s,
                              int wbits);
size_t wide_build_scratch_bytes(int nb, int wbits);
size_t fbw_words_per_base(int wbits);
// wave priority table (helpers.hpp PrioSlot) of rp_kernels.hip and msm.hip's kernels
hipError_t rp_set_wave_prio(const int* p);
extern std::atomic<int> g_work_bs;  // rp_kernels.hip (FTS_WORK_BS)
hipError_t msm_set_wave_prio(const int* p);
void launch_rp_fallback(const RpBatchDev& d, const uint32_t* tables, const int32_t* sel, int nsel, hipStream_t s,
                        Timeline* tl);
void launch_rlc_group_test(const RpBatchDev& d, const RlcDev& r, const uint32_t* tables, const MsmPlan& p,
                           const int32_t* sel, int G, int gs, uint32_t* gcol, uint32_t* gfix, int32_t* next,
                           uint32_t* next_count, hipStream_t s, Timeline* tl);
void launch_rp_gather(const RpGather& g, int k, uint8_t* raw, uint32_t* sc, int32_t* status, int32_t* ipa, hipStream_t s);
void launch_rlc_locate(const RpBatchDev& d, const RlcDev& r, const uint32_t* tables, uint32_t* save, int32_t* loc,
                       hipStream_t s, Timeline* tl);
void launch_rlc_accept_except(int B, int skip, int32_t* status, const int32_t* ipa_flag, hipStream_t s);
// ev_stage (optional): recorded on s after the counting sort (stage 1) or the bucket
// accumulation (stage 2)
void launch_msm(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra, int nextra,
                uint32_t* scratch, hipStream_t s, hipStream_t s_extra, Timeline* tl, hipEvent_t ev_stage = nullptr,
                int stage = 0);
void launch_msm_load(int N, const uint8_t* raw_pts, const uint8_t* raw_sc, uint32_t* pts, uint32_t* sc, uint32_t* bad,
                     hipStream_t s);
void launch_msm_to_bytes(const uint32_t* jac, uint8_t* out, hipStream_t s);
void launch_msm_pts_to_bytes(int n, const uint32_t* pts, uint8_t* out, hipStream_t s);
void launch_msm_gen_points(int N, const uint8_t* raw_k, const uint8_t* raw_s, const uint32_t* table, uint32_t* jac,
                           uint32_t* pts, uint32_t* sc, hipStream_t s);
void launch_sig_prep(const SigBatchDev& d, hipStream_t s);
void launch_sig_finish(const SigBatchDev& d, const uint32_t* tables, int n, hipStream_t s);
void launch_sig_exclude(const SigBatchDev& d, int32_t* rp_excl, hipStream_t s);
size_t table_build_scratch_bytes(int nb);
size_t fb_words_per_base();
// prove_kernels.hip
void launch_rp_prove(const PvDev& d, const PvStage* stages, const uint8_t* x0_const, const uint8_t* x0_tmpl,
                     hipStream_t s, Timeline* tl);
void launch_sigma_prove(const SpDev& d, hipStream_t s);
// audit_kernels.hip
void launch_open_check(int n, const uint8_t* raw, const uint32_t* sc, const uint32_t* tables, int nb,
                       int32_t* status, hipStream_t s);
}  // namespace fts

namespace fts {
// "fb:" + nm, interned (Timeline marks after fallback())
const char* fallback_name(const char* nm) {
  static std::mutex mu;
  static std::deque<std::string> names;  // stable storage (deque never moves elements)
  std::lock_guard<std::mutex> g(mu);
  const std::string want = std::string("fb:") + nm;
  for (const std::string& x : names)
    if (x == want) return x.c_str();
  names.push_back(want);
  return names.back().c_str();
}
}  // namespace fts

using namespace fts;
using namespace fts::host;

#define HIP_OK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "fts_gpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return FTS_API_EDEVICE;                                                             \
    }                                                                                     \
  } while (0)

namespace {

// growable device buffer
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  // grows geometrically: hipFree synchronises the whole device, so a buffer
  // must not be re-allocated on every slightly larger batch
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) hipFree(p);
    p = nullptr;
    const size_t grown = cap + cap / 2;
    cap = 0;
    size_t want = std::max<size_t>(std::max(bytes, grown), 256);
    if (hipMalloc(&p, want) != hipSuccess) return -1;
    cap = want;
    return 0;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

struct Workspace {
  DBuf pts, ch, small, hpj, hpa, hpbe, x0, x0mid, terms, scratch, ypow, svec, zvec, rp_excl;
  // random-linear-combination check + MSM
  DBuf r_key, r_msc, r_coef, r_colsum, r_fixed, r_flag, r_gcol, r_gfix, r_sel, r_next, r_cnt, m_keys,
      m_counts, m_offsets, m_cursor, m_sorted, m_buckets, m_segs, m_wins, m_out, m_scratch, m_win, m_choff, m_chbkt, m_partials;
  DBuf r_msel, r_mcol, r_mfix, r_mqfix, r_mflag;  // the per-caller-batch combination of a coalesced pass
  DBuf r_loc, r_save;  // the single-fault locator: located proof, the failed combination S
  // action (transfer / issue) batches
  DBuf rp_raw, rp_sc, rp_status, rp_ipa;
  DBuf s_act, s_raw, s_owner, s_pts, s_sc, s_status, s_work, s_terms, s_aff, s_affoff, s_msgs, s_jac, s_scratch;
  DBuf open_rec;  // token opening checks: [raw n*64][scalars n*96][status n*4]
  DBuf pv;        // batched prover: one arena (prove_arena)
  DBuf sp;        // sigma provers: one arena
  void release() {
    for (DBuf* b : {&open_rec, &pv, &sp, &pts, &ch, &small, &hpj, &hpa, &hpbe, &x0, &x0mid, &terms, &scratch, &ypow, &svec, &zvec, &rp_excl, &rp_raw, &rp_sc, &m_choff, &m_chbkt, &m_partials,
                    &rp_status, &rp_ipa, &s_act, &s_raw, &s_owner, &s_pts, &s_sc, &s_status, &s_work, &s_terms, &s_aff,
                    &s_affoff, &s_msgs, &s_jac, &s_scratch, &r_key, &r_msc, &r_coef, &r_colsum, &r_fixed, &r_flag, &r_gcol, &r_gfix,
                    &r_sel, &r_next, &r_cnt, &r_msel, &r_mcol, &r_mfix, &r_mqfix, &r_mflag, &r_loc, &r_save,
                    &m_keys, &m_counts, &m_offsets, &m_cursor, &m_sorted, &m_buckets, &m_segs, &m_wins, &m_out,
                    &m_scratch, &m_win})
      b->release();
  }
};


}  // namespace

// One execution lane: a main + side stream pair with its own workspace and
// timeline.  Independent batches submitted concurrently (e.g. by the Go shim's
// aggregation goroutines, or bench.py's pipeline) run on different lanes, so
// one batch's latency-bound phases (transcript hashing, doubling chains)
// overlap another batch's throughput-bound kernels.

// pinned window-table slots of Lane::Pinned (msm_prepare_plan)
enum { MSM_SLOT_PASS = 0, MSM_SLOT_RESERVE, MSM_SLOT_GT_BIG, MSM_SLOT_GT_SMALL, MSM_WIN_SLOTS };

struct Lane {
  int id = 0;
  // completion event created with hipEventBlockingSync: waiting on it sleeps
  // instead of spinning (a spinning waiter per lane burns the process's CPU
  // quota; on a CFS-throttled box that stalls every host thread for ~50 ms
  // out of each 100 ms period)
  hipEvent_t done = nullptr;
  hipError_t sync() {
    hipError_t e = hipEventRecord(done, s);
    return e == hipSuccess ? hipEventSynchronize(done) : e;
  }
  bool presized = false;  // workspace sized for the context's largest coalesced pass
  // no other pass was running when the current one started (set by the dispatchers):
  // only then does a small pass take the latency path (k_rp_fixed_all), which does
  // more total work than the work path and pays off only on an otherwise idle device
  bool alone = true;
  hipStream_t s = nullptr, s2 = nullptr;
  hipStream_t s3 = nullptr;         // sigma proofs of action batches (beside the range-proof pass)
  hipStream_t s4 = nullptr;         // the batch check's x0-free columns beside its MSM
  hipEvent_t ev_a = nullptr, ev_b = nullptr, ev_c = nullptr, ev_d = nullptr, ev_e = nullptr;  // cross-stream ordering (no timing)
  Workspace ws;
  Timeline tl;
  float host_prep_ms = 0, host_enqueue_ms = 0, host_wait_ms = 0;  // host wall time of the last run
  float host_parse_ms = 0, host_stage_ms = 0;  // action batches: DER parsing, assembly + upload
  float host_misc_ms = 0, host_total_ms = 0, host_stage_copy_ms = 0;  // action batches: allocation before the parse + verdict assembly / release after the wait
  // pinned host staging (pageable async copies would block the enqueue)
  struct Pinned {
    uint32_t key[8];
    // window tables of the MSM plans uploaded between two syncs of the lane
    // (msm_prepare_plan's `slot`): the group test uploads two plans back to
    // back, and one shared pinned source let the second memcpy overwrite the
    // first before its DMA ran
    MsmWindow win[MSM_WIN_SLOTS][MSM_MAX_WINDOWS];
    int32_t flag;
    int32_t gflag[RP_GATHER_MAX];  // per caller batch of a grouped pass: its combination closed
  }* pin = nullptr;
  int32_t* pin_status = nullptr;
  size_t pin_status_cap = 0;
  // action batches: pinned staging of the assembled sigma / range-proof inputs
  uint8_t* stage = nullptr;
  size_t stage_cap = 0;
  uint8_t* stage_buf(size_t bytes) {
    if (bytes > stage_cap) {
      if (stage) (void)hipHostFree(stage);
      stage = nullptr;
      const size_t want = std::max<size_t>(std::max(bytes, stage_cap + stage_cap / 2), 1 << 20);
      stage_cap = 0;
      if (hipHostMalloc((void**)&stage, want, 0) != hipSuccess) return nullptr;
      stage_cap = want;
    }
    return stage;
  }
  // pinned source of the per-caller-batch slot map (its own buffer: `stage` may still
  // be the source of an action batch's pending uploads)
  int32_t* pin_sel = nullptr;
  size_t pin_sel_cap = 0;
  int32_t* sel_buf(size_t n) {
    if (n > pin_sel_cap) {
      if (pin_sel) (void)hipHostFree(pin_sel);
      pin_sel = nullptr;
      pin_sel_cap = 0;
      const size_t want = std::max<size_t>(n, 1 << 16);
      if (hipHostMalloc((void**)&pin_sel, want * 4, 0) != hipSuccess) return nullptr;
      pin_sel_cap = want;
    }
    return pin_sel;
  }
  int32_t* status_buf(size_t n) {
    if (n > pin_status_cap) {
      if (pin_status) (void)hipHostFree(pin_status);
      pin_status = nullptr;
      pin_status_cap = 0;
      if (hipHostMalloc((void**)&pin_status, std::max<size_t>(n, 4096) * 4, 0) != hipSuccess) return nullptr;
      pin_status_cap = std::max<size_t>(n, 4096);
    }
    return pin_status;
  }
  void free_pinned() {
    if (pin) (void)hipHostFree(pin);
    if (pin_status) (void)hipHostFree(pin_status);
    if (pin_sel) (void)hipHostFree(pin_sel);
    pin_sel = nullptr;
    pin_sel_cap = 0;
    if (stage) (void)hipHostFree(stage);
    pin = nullptr;
    pin_status = nullptr;
    pin_status_cap = 0;
    stage = nullptr;
    stage_cap = 0;
  }
};
// host worker threads for batch parsing: the CPUs this process may actually
// use (cgroup v2 cpu.max quota, else the hardware count), at most 16
static unsigned host_threads() {
  static const unsigned n = [] {
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long period = 0;
      if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
        hw = std::min<unsigned>(hw, (unsigned)std::max(1LL, atoll(q) / period));
      fclose(f);
    }
    return std::min(16u, hw);
  }();
  return n;
}

// Fork-join pool of host_threads() - 1 persistent workers for the host loops
// (DER parsing, staging): spawning host_threads() std::threads per loop cost
// ~0.5 ms per loop, twice per action call, with several calls in flight.
// Every caller works on its own job too, so concurrent callers always progress.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();  // never destroyed: workers may outlive static destructors
    return *p;
  }
  void run(size_t n, const std::function<void(size_t)>& f) {
    auto j = std::make_shared<Job>();
    j->n = n;
    j->f = &f;
    // items are claimed in chunks: one atomic claim and one completion count per
    // chunk, not per item (per-item counters bounced one cache line between every
    // worker: ~0.8 us of overhead per parsed action with 8 threads)
    j->grain = std::max<size_t>(1, std::min<size_t>(32, n / (8 * (size_t)host_threads())));
    {
      std::lock_guard<std::mutex> l(mu_);
      q_.push_back(j);
    }
    cv_.notify_all();
    work(*j);
    std::unique_lock<std::mutex> l(j->m);
    j->cv.wait(l, [&] { return j->done.load() == j->n; });
  }

 private:
  struct Job {
    size_t n = 0, grain = 1;
    const std::function<void(size_t)>* f = nullptr;
    std::atomic<size_t> next{0}, done{0};
    std::mutex m;
    std::condition_variable cv;
  };
  HostPool() {
    const unsigned nw = host_threads() > 1 ? host_threads() - 1 : 0;
    for (unsigned t = 0; t < nw; t++) std::thread([this] { loop(); }).detach();
  }
  static void work(Job& j) {
    for (size_t i0; (i0 = j.next.fetch_add(j.grain)) < j.n;) {
      const size_t i1 = std::min(j.n, i0 + j.grain);
      for (size_t i = i0; i < i1; i++) (*j.f)(i);
      if ((j.done += i1 - i0) == j.n) {
        std::lock_guard<std::mutex> l(j.m);
        j.cv.notify_all();
      }
    }
  }
  void loop() {
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return !q_.empty(); });
        j = q_.front();
        if (j->next.load() >= j->n) {  // exhausted: drop it and look again
          q_.pop_front();
          continue;
        }
      }
      work(*j);
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<Job>> q_;
};

// run f(i) for i in [0, n) on the host pool (inline when small)
template <class F>
static void parallel_for(size_t n, size_t min_parallel, F&& f) {
  if (n < min_parallel || host_threads() <= 1) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  const std::function<void(size_t)> fn = std::ref(f);
  HostPool::get().run(n, fn);
}
namespace fts {
// the same pool for the signature batches' packing loops (ecdsa_kernels.hip, idemix_kernels.hip)
void host_parallel_for(size_t n, const std::function<void(size_t)>& f) { parallel_for(n, 2, f); }
}  // namespace fts

static inline double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct ActSlot;
// One call waiting for (or being served by) a device pass: a staged range-proof
// batch (fts_rp_batch_verify, fts_rp_verify_batch), or an action call (transfers /
// issues / requests) whose range proofs are `b` and whose sigma batch is `act`.
struct RpReq {
  fts_rp_batch* b;
  int32_t* status;  // caller's host status array of b's proofs (may be null)
  ActSlot* act = nullptr;
  int rc = 0;
  bool done = false;
  std::chrono::steady_clock::time_point arrived = std::chrono::steady_clock::now();
  std::condition_variable cv;  // this caller's wake-up (targeted, no thundering herd)
  RpReq(fts_rp_batch* bb, int32_t* st, ActSlot* a = nullptr) : b(bb), status(st), act(a) {}
};

namespace {
struct ActionIn {
  int kind;                    // SIG_TAS / SIG_ST
  const uint8_t* in;           // n_in * 64
  size_t n_in;
  const uint8_t* out;          // n_out * 64 (issue: tokens)
  size_t n_out;
  der::Span proof;
};

struct ActionState {
  int32_t host_final = -1;     // verdict decided on the host (MALFORMED / TAS_INVALID)
  int sig = -1;                // index in the call's sigma batch (-1: decided before the layout)
  bool rc_applicable = false;
  int rp_base = -1, rp_count = 0;
  bool rc_count_bad = false;
};
}  // namespace

// An action call staged for the dispatcher (act_stage), pooled per context like
// RpSlot: the call's records parsed straight into pinned host memory in their
// device layout, one upload into `dev`, and the call's sigma workspace behind
// them in `dev`.  Its sigma proofs (TypeAndSum / SameType, independent of the
// range proofs) run at once on the slot's own stream, while the call waits for a
// pass; they also write the V slots of its range proofs.  A device pass then
// verifies the range proofs of several calls as one batch (gathered like staged
// range-proof batches) after the calls' sigma events, so concurrent transfer /
// issue / request calls share passes instead of taking a lane each, and the sigma
// work overlaps other passes instead of sitting on a pass's critical path
// (DESIGN.md §3.4).
struct ActSlot {
  fts_rp_batch* b = nullptr;  // the call's range proofs: raw / sc / status0 / ipa point into `dev`
  uint8_t* pin = nullptr;
  size_t pin_cap = 0;
  uint8_t* dev = nullptr;
  size_t dev_cap = 0;
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;   // blocking-sync: the staging caller sleeps
  // on s: [0] before the sigma kernels, [1] after decode + primes + V slots, [2] after
  // the sigma equations (the pass waits for it before gathering the range proofs)
  hipEvent_t ev_sig[3] = {nullptr, nullptr, nullptr};
  SigBatchDev sd{};            // the call's sigma batch (sd.A == 0: none); rp_raw = the slot's range proofs
  int32_t* sig_res = nullptr;  // pinned: sigma verdicts [sd.A], downloaded by the pass
  std::vector<int32_t> rp_res;  // range-proof verdicts [b->B], scattered by the pass
  std::vector<ActionState> st;
  std::vector<uint8_t> host_buf;  // host-only contexts: the records (no device)
  float parse_ms = 0, stage_ms = 0;
  float phase_ms[3] = {0, 0, 0};  // act_stage's shapes / layout / decode steps of the last call
};

// fts_rp_verify_batch staging slot (host DER bytes -> device): pinned host
// records and device input buffers, grown geometrically and reused across
// calls, so a call neither allocates nor frees device memory (hipFree
// synchronises the whole device, stalling every other lane's pass)
struct RpSlot {
  fts_rp_batch* b = nullptr;  // device pointers into `dev` (not owned by the batch)
  uint8_t* pin = nullptr;
  size_t pin_cap = 0;
  uint8_t* dev = nullptr;
  size_t dev_cap = 0;
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;  // blocking-sync: the waiting caller sleeps
};

struct fts_ctx {
  int device = 0;
  // multi-device context (fts_ctx_create_devices): one child context per device;
  // batch entry points shard their batch over the children (multi_* below)
  std::vector<fts_ctx*> shards;
  PublicParams pp;
  int n = 0, k = 0;
  uint32_t* d_tables = nullptr;
  uint32_t* d_wtables = nullptr;  // wide tables of [H_0 .. H_{n-1}, K, P] (k_rp_fixed_exact)
  // their window width: 22 bits (12 additions per product, 1.5 GiB per base) when the
  // device has the memory at context creation, else 20 (13, 436 MiB); FTS_WIDE_BITS
  int wbits = 20;
  int wbits_forced = 0;  // fts_ctx_opts.wide_bits / FTS_WIDE_BITS: no fallback to 20 bits
  int nlanes = 0;
  uint8_t* d_x0const = nullptr;
  uint8_t* d_x0tmpl = nullptr;  // x0 message blocks [x0_cb0, x0_cb1): shared by every proof
  size_t table_bytes = 0;
  // lane pool
  std::vector<Lane*> lanes;
  std::vector<int> free_lanes;
  std::mutex mu;
  std::condition_variable cv;
  int last_lane = 0;
  // timings of the most recently completed range-proof run
  std::mutex tim_mu;
  int ntim = 0;
  const char* tim_name[Timeline::CAP];
  float tim_ms[Timeline::CAP];
  double tim_work[Timeline::CAP];
  std::atomic<int> last_fallback{0};
  // batch coalescing (fts_rp_batch_verify): staged batches submitted
  // concurrently are merged into one device pass of up to coalesce_max proofs
  std::deque<RpReq*> rp_pending;
  size_t pending_proofs = 0;  // proofs queued in rp_pending
  // 81,920 proofs (20 batches of 4,096): a burst of batches (the driver's 20-step
  // bench) shares two or three large passes, whose chain kernels (com, the
  // per-proof x0 hash, the MSM's final reduction) run at several waves per SIMD
  // instead of under one (tools/s20_sweep4.sh: 3.0 -> 3.6 M rp64/s at 20 steps,
  // 4.41 -> 4.47 M/s at 512 steps, single-batch latency unchanged)
  size_t coalesce_max = 81920;
  // gather window: while the device is busy and fewer than gather_target proofs
  // are queued, the head request waits up to gather_us for more batches before
  // it takes a lane (a burst of callers then shares a few large passes instead
  // of one lone 4,096-proof pass per free lane); an idle device starts at once
  size_t gather_target = 16384;
  int gather_us = 1000;
  // An idle device's window (FTS_IDLE_GATHER_US / FTS_IDLE_QUIET_US): the head waits
  // while batches keep arriving (each within idle_quiet_us of the last, at most
  // idle_gather_us in all) or until gather_target proofs are queued, and its pass
  // takes at most gather_target proofs.  A burst of 20 callers released together
  // (the driver's 20-step line) becomes two passes of 10 batches whatever the
  // threads' timing (r05: 4.19-4.32 M/s medians with passes of 1 + 10 + 9, formed by
  // arrival luck; 4.35-4.40 with 10 + 10); a lone caller waits idle_quiet_us.
  int idle_gather_us = 1000;
  int idle_quiet_us = 150;
  std::chrono::steady_clock::time_point last_arrival{};
  // FTS_IDLE_FIRST_US: a caller that arrives at an idle device with no other arrival in
  // the last idle_quiet_us (a lone caller, not part of a burst) waits only this long
  // for company -- spinning, not on a condition variable whose wake-up alone cost
  // ~0.1 ms -- and starts at once when nobody comes (round 5 paid the whole quiet gap
  // plus a wake-up: 3.36 vs 2.75-2.86 ms for a lone 4,096-proof batch)
  int idle_first_us = 30;
  std::atomic<uint64_t> arrivals{0};
  // test hook (fts_debug_hold): no pass starts until hold_n requests are queued
  int hold_n = 0;
  // dispatcher counters (fts_debug_dispatch_stats)
  std::atomic<int64_t> st_passes{0}, st_reqs{0}, st_max_merged{0}, st_act_reqs{0};
  // passes of up to com_fixed_max proofs compute com on the latency path (fixed-base
  // groups, rp_kernels.hip k_rp_fixed_all), larger ones on the work path (Horner +
  // joint GLV chains): the same group element either way
  size_t com_fixed_max = 16384;
  // group test: round-1 group size and round-2 threshold (FTS_GT1 / FTS_GT2_MIN).  Larger
  // round-1 groups make the grouped MSM's bucket reduction cheaper (it scales with the
  // group count); the per-proof checks of the failing groups cost one GLV chain of
  // latency whatever their number up to ~8k proofs (tools/gt_sweep.sh, C5 1 % tampered:
  // 64/2048 -> 256/8192 = 485k -> 533k actions/s)
  int gt1 = 256, gt2_min = 8192;
  // FTS_LOCATE: after a failed (ungrouped) batch check whose caller batches are all
  // sparse, first the single-fault locator (rp_locate_single): one index-weighted
  // recombination + a lane per proof, instead of the group test's grouped MSM
  bool locate = true;
  // after a miss (several bad proofs) each caller batch of the pass that holds a bad
  // proof skips the locator in its next locate_backoff failing passes, the backoff
  // doubling per consecutive miss (8 .. 256) and reset by a hit: a stream of
  // multi-fault batches (C5, tampered C2) pays it rarely.  Kept per caller batch
  // (fts_rp_batch::locate_skip), so one caller's multi-fault passes never make
  // another caller's single-fault passes skip the locator
  // action calls (transfer / issue / mixed / request) have no batch object across
  // calls: they share one locator backoff, carried into each call's slot batch and
  // back (a stream of multi-fault calls -- C5 with 1 % tampered actions -- would
  // otherwise pay a missed locator, one extra MSM, on every call)
  std::atomic<int> act_locate_skip{0}, act_locate_backoff{8};
  // FTS_GT_ADAPT: a staged caller batch's round-1 group size follows the bad-proof
  // density of ITS last failed verification (fts_rp_batch::dense; per caller batch,
  // so one caller's tampered batches never change the fallback of another's).
  // Dense (more than half the batch's proofs in failing 256-groups, or more than
  // 2 % in failing 8-groups: ~0.3 % bad proofs and up) starts at groups of 8 on the
  // small-group kernels; a 256-group round there is one whole grouped Pippenger MSM
  // that clears almost nothing (C2 with 1 % tampered, 81,920-proof pass: 51.8 ->
  // 41.4 ms; C5's sparse bad proofs keep 256, where 8 was slower,
  // tools/sweeps/gt1_small.txt).  Action calls have no batch across calls: 256.
  int gt_adapt = 1;
  // FTS_X0_SPLIT: bit 0 the work path hashes the x0 prefix beside the com chain, bit 1
  // the latency path beside com_tree (round 6: a lone 4,096-proof batch 3.15 -> 2.87 ms,
  // profiles/r06_x0_split_ab/); 1 = the work path only (rounds 2-5)
  int x0_split = 3;
  // FTS_MSM_SORT: the MSMs' two-level counting sort (msm.hip k_rs_*; 0: k_msm_digits'
  // device atomics + k_msm_scatter, the round-4 batch-check sort, for A/B)
  int msm_sort = 1;
  // FTS_MSM_MAXC: the widest MSM window this context's plans take (per context: one
  // context's setting never changes another's plans)
  int msm_maxc = 16;
  // FTS_MAIN_GROUPS=1: a coalesced pass checks one random linear combination PER CALLER
  // BATCH (a G-group MSM + per-group column sums), so a bad proof's fallback covers
  // its own batch only.  Default 0 (one combination over the pass): the grouped MSM's
  // extra windows and per-group bucket reductions cost 10-17 % of the clean 512-step
  // rate (4.96 -> 4.47 M rp64/s, gpurun_out/r05b) for +10 % with one bad proof per pass
  int main_groups = 0;
  // FTS_FX_SERIAL: passes' fixed-base launches run one at a time across the lanes
  // (device-side event chain under fx_mu), staggering concurrent passes
  int fx_serial = 0;
  std::mutex fx_mu;
  hipEvent_t fx_last = nullptr;  // the fixed-base event of the pass enqueued last
  // FTS_RLC_FORK: the batch check forks after the fixed-base products (1) or after the
  // challenges (0); 2 (default): after the challenges on the latency path (a lone small
  // pass: its MSM chain is the critical path, 3.16 -> 2.98 ms per 4,096-proof batch),
  // after the fixed-base products on the work path (larger passes: 4.69 -> 4.82 M/s at
  // 512 steps; tools/run_lat4k.sh, tools/run_fork.sh)
  int rlc_fork = 2;
  // a lane was freed (call with mu held): the head pending range-proof request
  // becomes the next leader; LaneGuard waiters re-check too
  void wake_lane_waiters() {
    if (!rp_pending.empty()) rp_pending.front()->cv.notify_one();
    cv.notify_all();
  }
  std::once_flag prover_once;
  ProverTables ptab;
  std::mutex slot_mu;
  std::vector<RpSlot*> slots, free_slots;  // fts_rp_verify_batch staging (all / idle)
  std::vector<ActSlot*> aslots, free_aslots;  // action-call staging (all / idle), under slot_mu
};

// RAII lane acquisition (want < 0: any free lane)
struct LaneGuard {
  fts_ctx* c;
  Lane* L;
  LaneGuard(fts_ctx* cc, int want = -1) : c(cc), L(nullptr) {
    std::unique_lock<std::mutex> lk(c->mu);
    c->cv.wait(lk, [&] {
      if (want < 0) return !c->free_lanes.empty();
      return std::find(c->free_lanes.begin(), c->free_lanes.end(), want) != c->free_lanes.end();
    });
    auto it = want < 0 ? c->free_lanes.end() - 1 : std::find(c->free_lanes.begin(), c->free_lanes.end(), want);
    L = c->lanes[*it];
    c->free_lanes.erase(it);
    L->alone = c->free_lanes.size() + 1 == c->lanes.size();
  }
  ~LaneGuard() {
    std::lock_guard<std::mutex> lk(c->mu);
    c->free_lanes.push_back(L->id);
    c->wake_lane_waiters();
  }
};

struct fts_rp_batch {
  int B = 0;
  int device = 0;
  // staged on a multi-device context: one child batch per shard, shard j holds
  // proofs [bounds[j], bounds[j+1]) of the caller's batch
  std::vector<fts_rp_batch*> parts;
  std::vector<fts_ctx*> part_ctx;
  std::vector<size_t> bounds;
  int merged = 1;  // batches in the device pass that verified it last
  bool dense = false;  // its last failed verification found dense bad proofs (FTS_GT_ADAPT)
  int locate_skip = 0, locate_backoff = 8;  // single-fault locator backoff (fts_ctx::locate)
  // timings of this batch's last verification
  int ntim = 0;
  const char* tim_name[Timeline::CAP];
  float tim_ms[Timeline::CAP];
  double tim_work[Timeline::CAP];
  uint8_t* raw = nullptr;
  uint32_t* sc = nullptr;
  int32_t* status0 = nullptr;  // host-parse verdicts (restored before every run)
  int32_t* status = nullptr;
  int32_t* ipa_flag = nullptr;
};

namespace fts {
namespace host {
void build_prover_tables(const PublicParams& pp, int n, ProverTables& t) {
  t.n = n;
  std::vector<G1A> bases;
  for (int i = 0; i < n; i++) bases.push_back(pp.left[i]);
  for (int i = 0; i < n; i++) bases.push_back(pp.right[i]);
  for (int i = 0; i < 3; i++) bases.push_back(pp.ped[i]);
  bases.push_back(pp.P);
  bases.push_back(pp.Q);
  t.fb.resize(bases.size());
  std::atomic<size_t> next{0};
  unsigned nth = host_threads();
  std::vector<std::thread> th;
  for (unsigned w = 0; w < nth; w++)
    th.emplace_back([&]() {
      for (size_t i; (i = next++) < bases.size();) t.fb[i].build(bases[i]);
    });
  for (auto& x : th) x.join();
}
}  // namespace host
}  // namespace fts

static int ctx_create(const uint8_t* pp_bytes, size_t pp_len, uint32_t bits, int device, fts_ctx** out,
                      const fts_ctx_opts* opts = nullptr) {
  if (!pp_bytes || !out) return FTS_API_EINVAL;
  *out = nullptr;
  fts_ctx* c = new fts_ctx();
  std::string err;
  if (!parse_public_params(pp_bytes, pp_len, c->pp, err)) {
    fprintf(stderr, "fts_gpu: public parameters rejected: %s\n", err.c_str());
    delete c;
    return FTS_API_EPP;
  }
  if (bits) {
    if (bits > c->pp.bit_length || (bits & (bits - 1)) || bits < 2) {
      delete c;
      return FTS_API_ESIZE;
    }
    c->pp.left.resize(bits);
    c->pp.right.resize(bits);
    c->pp.bit_length = bits;
    c->pp.rounds = 63 - __builtin_clzll(bits);
    c->pp.max_token = bits == 64 ? ~0ULL : ((1ULL << bits) - 1);
    c->pp.precision = bits;
  }
  c->n = (int)c->pp.bit_length;
  c->k = (int)c->pp.rounds;
  if (device == FTS_DEVICE_NONE) {  // host-only context: parsing + prover, no GPU
    c->device = FTS_DEVICE_NONE;
    *out = c;
    return FTS_API_OK;
  }
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) device = 0;
  }
  c->device = device;
  auto fail = [&](int code) {
    for (Lane* L : c->lanes) {
      if (L->s3) hipStreamDestroy(L->s3);
      if (L->ev_a) hipEventDestroy(L->ev_a);
      if (L->ev_b) hipEventDestroy(L->ev_b);
      if (L->ev_c) hipEventDestroy(L->ev_c);
      if (L->ev_d) hipEventDestroy(L->ev_d);
      if (L->ev_e) hipEventDestroy(L->ev_e);
      if (L->s2 && L->s2 != L->s) hipStreamDestroy(L->s2);
      if (L->s4 && L->s4 != L->s) hipStreamDestroy(L->s4);
      if (L->s) hipStreamDestroy(L->s);
      L->tl.destroy();
      if (L->done) hipEventDestroy(L->done);
      L->free_pinned();
      delete L;
    }
    if (c->d_tables) hipFree(c->d_tables);
    if (c->d_wtables) hipFree(c->d_wtables);
    delete c;
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(FTS_API_EDEVICE);
  int nl = 4;  // lanes (FTS_LANES): 4 beat 5 and 3 on the burst and the steady state (s20_sweep4.sh)
  if (const char* e = getenv("FTS_LANES")) nl = std::max(1, std::min(16, atoi(e)));
  if (opts && opts->lanes > 0) nl = std::min(16, opts->lanes);
  c->nlanes = nl;
  if (const char* e = getenv("FTS_COALESCE_MAX")) c->coalesce_max = (size_t)std::max(0L, atol(e));
  c->gather_target = c->coalesce_max / 2;
  if (const char* e = getenv("FTS_GATHER_TARGET")) c->gather_target = (size_t)std::max(1L, atol(e));
  if (const char* e = getenv("FTS_GATHER_US")) c->gather_us = std::max(0, atoi(e));
  if (const char* e = getenv("FTS_IDLE_GATHER_US")) c->idle_gather_us = std::max(0, atoi(e));
  if (const char* e = getenv("FTS_IDLE_QUIET_US")) c->idle_quiet_us = std::max(0, atoi(e));
  if (const char* e = getenv("FTS_IDLE_FIRST_US")) c->idle_first_us = std::max(0, atoi(e));
  if (const char* e = getenv("FTS_COM_FIXED_MAX")) c->com_fixed_max = (size_t)std::max(0L, atol(e));
  if (const char* e = getenv("FTS_RLC_FORK")) c->rlc_fork = std::max(0, std::min(4, atoi(e)));
  if (const char* e = getenv("FTS_X0_SPLIT")) c->x0_split = std::max(0, std::min(3, atoi(e)));
  if (const char* e = getenv("FTS_MSM_SORT")) c->msm_sort = atoi(e) != 0;
  if (const char* e = getenv("FTS_MAIN_GROUPS")) c->main_groups = atoi(e) != 0;
  if (const char* e = getenv("FTS_FX_SERIAL")) c->fx_serial = atoi(e) != 0;
  {  // process-wide, like the priority table: every context sets it (the last one wins)
    const char* e = getenv("FTS_WORK_BS");
    g_work_bs.store(e && atoi(e) == 256 ? 256 : 64, std::memory_order_relaxed);
  }
  if (const char* e = getenv("FTS_GT1")) c->gt1 = std::max(8, std::min(1024, atoi(e)));
  if (const char* e = getenv("FTS_GT2_MIN")) c->gt2_min = std::max(0, atoi(e));
  if (const char* e = getenv("FTS_GT_ADAPT")) c->gt_adapt = atoi(e) != 0;
  if (const char* e = getenv("FTS_LOCATE")) c->locate = atoi(e) != 0;
  if (const char* e = getenv("FTS_MSM_MAXC")) c->msm_maxc = std::max(8, std::min(16, atoi(e)));
  // FTS_WAVE_PRIO: one digit 0-3 per PrioSlot (device/wave_prio.hpp), e.g.
  // 022113313133; the table is per device and process: every context uploads its
  // own (the default without the variable), the last one created on a device wins
  {
    int pr[PS_N] = FTS_WAVE_PRIO_DEFAULT;
    if (const char* e = getenv("FTS_WAVE_PRIO"))
      for (int i = 0; i < PS_N && e[i]; i++)
        if (e[i] >= '0' && e[i] <= '3') pr[i] = e[i] - '0';
    if (rp_set_wave_prio(pr) != hipSuccess || msm_set_wave_prio(pr) != hipSuccess) return fail(FTS_API_EDEVICE);
  }
  // the batch check's stream (s3: RLC weights + MSM, the longest chain of a small
  // pass) gets the device's highest stream priority, so its few waves are
  // dispatched ahead of the exact phase's wide fixed-base launches
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
  for (int i = 0; i < nl; i++) {
    Lane* L = new Lane();
    L->id = i;
    c->lanes.push_back(L);
    c->free_lanes.push_back(i);
    if (hipStreamCreateWithFlags(&L->s, hipStreamNonBlocking) != hipSuccess) return fail(FTS_API_EDEVICE);
    if (hipEventCreateWithFlags(&L->done, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess)
      return fail(FTS_API_EDEVICE);
    if (hipHostMalloc((void**)&L->pin, sizeof(Lane::Pinned), 0) != hipSuccess) return fail(FTS_API_ENOMEM);
    if (hipStreamCreateWithFlags(&L->s2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&L->s4, hipStreamNonBlocking) != hipSuccess)
      return fail(FTS_API_EDEVICE);
    if (hipStreamCreateWithPriority(&L->s3, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipEventCreateWithFlags(&L->ev_a, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&L->ev_b, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&L->ev_c, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&L->ev_d, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&L->ev_e, hipEventDisableTiming) != hipSuccess)
      return fail(FTS_API_EDEVICE);
    L->tl.create();
  }
  hipStream_t s0 = c->lanes[0]->s;
  const int n = c->n;
  // fixed bases in table order (rp_kernels.hpp tb_*)
  std::vector<G1A> bases;
  for (int i = 0; i < n; i++) bases.push_back(c->pp.left[i]);
  for (int i = 0; i < n; i++) bases.push_back(c->pp.right[i]);
  bases.push_back(c->pp.ped[1]);
  bases.push_back(c->pp.ped[2]);
  bases.push_back(c->pp.P);
  bases.push_back(c->pp.Q);
  G1J K = jac_identity();
  for (int i = 0; i < n; i++) {
    K = jadd_aff(K, c->pp.right[i]);
    K = jadd_aff(K, aff_neg(c->pp.left[i]));
  }
  bases.push_back(to_aff(K));
  bases.push_back(c->pp.ped[0]);
  const int nb = (int)bases.size();
  std::vector<uint32_t> hb((size_t)nb * 16, 0);
  for (int b = 0; b < nb; b++)
    if (!bases[b].inf) {
      memcpy(&hb[b * 16], bases[b].x.v, 32);  // 4x64 LE == 8x32 LE Montgomery form
      memcpy(&hb[b * 16 + 8], bases[b].y.v, 32);
    }
  uint32_t* d_bases = nullptr;
  uint32_t* d_scr = nullptr;
  c->table_bytes = (size_t)nb * fb_words_per_base() * 4;
  if (hipMalloc(&c->d_tables, c->table_bytes) != hipSuccess) return fail(FTS_API_ENOMEM);
  if (hipMalloc(&d_bases, hb.size() * 4) != hipSuccess) return fail(FTS_API_ENOMEM);
  const int chunk = std::min(nb, 16);  // bases per build pass (bounds the Jacobian scratch)
  if (hipMalloc(&d_scr, table_build_scratch_bytes(chunk)) != hipSuccess) {
    hipFree(d_bases);
    return fail(FTS_API_ENOMEM);
  }
  hipMemcpyAsync(d_bases, hb.data(), hb.size() * 4, hipMemcpyHostToDevice, s0);
  for (int b0 = 0; b0 < nb; b0 += chunk)
    launch_build_tables(d_bases + (size_t)b0 * 16, std::min(chunk, nb - b0), c->d_tables + (size_t)b0 * fb_words_per_base(),
                        d_scr, s0);
  // wide tables of the per-proof bases H_i, K, P (same build, wider windows):
  // 22-bit windows (one mixed addition fewer per product: -8 % of the pass's
  // largest kernel) when the free HBM holds them with room to spare for the lanes'
  // workspace (~7 GB each at n = 64) and other contexts (160 GiB: at n = 64 only the
  // first context on an empty MI355X takes them); else, or when the allocation
  // fails, 20-bit
  {
    const int nw = n + 2;
    {
      // explicit width (fts_ctx_opts.wide_bits, else FTS_WIDE_BITS), else the budget:
      // 22-bit only when the whole context's tables fit the caller's table_budget
      // (fts_ctx_opts) or, without one, when the free HBM keeps every lane's
      // workspace (~8 GiB each for 81,920-proof passes at n = 64) and 128 GiB for
      // other contexts and processes on the device
      int wb = 20, forced = 0;
      if (opts && (opts->wide_bits == 20 || opts->wide_bits == 22)) {
        wb = opts->wide_bits, forced = 1;
      } else if (const char* e = getenv("FTS_WIDE_BITS")) {
        wb = atoi(e) == 22 ? 22 : 20, forced = 1;
      } else {
        size_t fr = 0, tot = 0;
        const size_t need22 = (size_t)nw * fbw_words_per_base(22) * 4;
        if (opts && opts->table_budget) {
          if (c->table_bytes + need22 <= opts->table_budget) wb = 22;
        } else if (hipMemGetInfo(&fr, &tot) == hipSuccess &&
                   fr > need22 + (size_t)nl * ((size_t)8 << 30) + ((size_t)128 << 30)) {
          wb = 22;
        }
      }
      c->wbits = wb;
      c->wbits_forced = forced;
    }
    std::vector<uint32_t> hw((size_t)nw * 16, 0);
    for (int i = 0; i < nw; i++) {
      const int src = i < n ? n + i : (i == n ? 2 * n + 4 : 2 * n + 2);  // H_i, K, P in `bases`
      memcpy(&hw[(size_t)i * 16], &hb[(size_t)src * 16], 64);
    }
    uint32_t* d_wb = nullptr;
    uint32_t* d_wscr = nullptr;
    int wchunk = 1;
    for (;;) {  // 22-bit tables that do not fit after all (other contexts' lanes): 20-bit
      wchunk = std::min(nw, c->wbits == 22 ? 1 : 4);  // bounds the Jacobian build scratch (2.4 / 1.6 GB)
      if (hipMalloc(&c->d_wtables, (size_t)nw * fbw_words_per_base(c->wbits) * 4) == hipSuccess &&
          hipMalloc(&d_wb, hw.size() * 4) == hipSuccess &&
          hipMalloc(&d_wscr, wide_build_scratch_bytes(wchunk, c->wbits)) == hipSuccess)
        break;
      if (d_wb) hipFree(d_wb);
      if (c->d_wtables) hipFree(c->d_wtables);
      d_wb = nullptr;
      c->d_wtables = nullptr;
      (void)hipGetLastError();
      if (c->wbits == 22 && !c->wbits_forced) {
        c->wbits = 20;
        continue;
      }
      hipFree(d_bases);
      hipFree(d_scr);
      return fail(FTS_API_ENOMEM);
    }
    hipMemcpyAsync(d_wb, hw.data(), hw.size() * 4, hipMemcpyHostToDevice, s0);
    for (int b0 = 0; b0 < nw; b0 += wchunk)
      launch_build_wide_tables(d_wb + (size_t)b0 * 16, std::min(wchunk, nw - b0),
                               c->d_wtables + (size_t)b0 * fbw_words_per_base(c->wbits), d_wscr, s0, c->wbits);
    c->table_bytes += (size_t)nw * fbw_words_per_base(c->wbits) * 4;
    hipError_t we = hipStreamSynchronize(s0);
    hipFree(d_wb);
    hipFree(d_wscr);
    if (we != hipSuccess) {
      hipFree(d_bases);
      hipFree(d_scr);
      return fail(FTS_API_EDEVICE);
    }
  }
  // constant part of the x0 transcript: hex(G_i) "||" ... hex(Q) "||"
  std::string xc;
  for (int i = 0; i <= n; i++) {
    uint8_t b[64];
    g1_to_bytes(i < n ? c->pp.left[i] : c->pp.Q, b);
    xc += hex_of(b, 64);
    xc += "||";
  }
  if (hipMalloc(&c->d_x0const, xc.size()) != hipSuccess) return fail(FTS_API_ENOMEM);
  hipMemcpyAsync(c->d_x0const, xc.data(), xc.size(), hipMemcpyHostToDevice, s0);
  // block-aligned template of the fully constant SHA-256 blocks of the x0 message
  std::string xt(64u * (x0_cb1(n) - x0_cb0(n)), '\0');
  for (size_t j = 0; j < xt.size(); j++) xt[j] = xc[64u * x0_cb0(n) + j - x0_const_off(n)];
  if (hipMalloc(&c->d_x0tmpl, xt.size()) != hipSuccess) return fail(FTS_API_ENOMEM);
  hipMemcpyAsync(c->d_x0tmpl, xt.data(), xt.size(), hipMemcpyHostToDevice, s0);
  hipError_t e = hipStreamSynchronize(s0);
  hipFree(d_bases);
  hipFree(d_scr);
  if (e != hipSuccess) {
    fprintf(stderr, "fts_gpu: table build failed: %s\n", hipGetErrorString(e));
    return fail(FTS_API_EDEVICE);
  }
  *out = c;
  return FTS_API_OK;
}

// ------------------------------------------------------ multi-device layer
// A context over several devices (fts_ctx_create_devices / _mask) owns one
// child context per device -- its own fixed-base tables, lanes, streams and
// workspace -- and parses the public parameters itself as a host-only context
// (host provers, commitments).  Each batch entry point splits the caller's
// batch into contiguous shards balanced by a cost weight (fts_shard_plan),
// runs shard j on child j from its own host thread, and lets every child write
// its verdicts straight into the caller's arrays at the shard's offset: the
// verdicts come back in caller order.  The reference verifies every action
// independently (core/common/validator.go:215-224), so no data crosses devices;
// each device closes its own random-linear-combination check.
extern "C" int fts_shard_plan(size_t n, const double* weights, int nshards, size_t* bounds) {
  if (nshards < 1 || !bounds) return FTS_API_EINVAL;
  double tot = 0;
  for (size_t i = 0; i < n; i++) tot += weights ? std::max(0.0, weights[i]) : 1.0;
  bounds[0] = 0;
  size_t i = 0;
  double acc = 0;
  for (int j = 1; j < nshards; j++) {
    const double target = tot * j / nshards;
    // first index whose prefix weight reaches the target (never behind the previous cut)
    while (i < n && acc + (weights ? std::max(0.0, weights[i]) : 1.0) * 0.5 <= target) {
      acc += weights ? std::max(0.0, weights[i]) : 1.0;
      i++;
    }
    bounds[j] = i;
  }
  bounds[nshards] = n;
  return FTS_API_OK;
}

// run f(j, lo, hi) for every non-empty shard j concurrently; first error wins
template <class F>
static int run_shards(const std::vector<size_t>& bnd, F&& f) {
  const int ns = (int)bnd.size() - 1;
  std::vector<int> rc(ns, FTS_API_OK);
  std::vector<std::thread> th;
  for (int j = 0; j < ns; j++)
    if (bnd[j + 1] > bnd[j]) th.emplace_back([&, j]() { rc[j] = f(j, bnd[j], bnd[j + 1]); });
  for (auto& t : th) t.join();
  for (int r : rc)
    if (r != FTS_API_OK) return r;
  return FTS_API_OK;
}
static std::vector<size_t> plan(size_t n, const std::vector<double>* w, int ns) {
  std::vector<size_t> b(ns + 1);
  fts_shard_plan(n, w ? w->data() : nullptr, ns, b.data());
  return b;
}

extern "C" {

int fts_ctx_create_devices(const uint8_t* pp, size_t pp_len, uint32_t bit_length, const int32_t* devices, int ndev,
                           fts_ctx** out) {
  if (!pp || !out || !devices || ndev < 1 || ndev > 64) return FTS_API_EINVAL;
  *out = nullptr;
  fts_ctx* c = nullptr;
  // the parent: parsed parameters, host-only (host provers / commitments run here)
  int rc = fts_ctx_create_bits(pp, pp_len, bit_length, FTS_DEVICE_NONE, &c);
  if (rc != FTS_API_OK) return rc;
  c->shards.assign(ndev, nullptr);
  std::vector<int> crc(ndev, FTS_API_OK);
  std::vector<std::thread> th;  // tables of every device built concurrently
  for (int j = 0; j < ndev; j++)
    th.emplace_back([&, j]() { crc[j] = fts_ctx_create_bits(pp, pp_len, bit_length, devices[j], &c->shards[j]); });
  for (auto& t : th) t.join();
  for (int j = 0; j < ndev; j++)
    if (crc[j] != FTS_API_OK) rc = crc[j];
  if (rc != FTS_API_OK) {
    fts_ctx_destroy(c);
    return rc;
  }
  c->device = c->shards[0]->device;
  *out = c;
  return FTS_API_OK;
}

int fts_ctx_create_mask(const uint8_t* pp, size_t pp_len, uint32_t bit_length, uint64_t device_mask, fts_ctx** out) {
  std::vector<int32_t> devs;
  for (int d = 0; d < 64; d++)
    if ((device_mask >> d) & 1u) devs.push_back(d);
  if (devs.empty()) return FTS_API_EINVAL;
  return fts_ctx_create_devices(pp, pp_len, bit_length, devs.data(), (int)devs.size(), out);
}

int fts_ctx_devices(const fts_ctx* c, int32_t* devices, int cap) {
  if (!c) return 0;
  if (c->shards.empty()) {
    if (devices && cap > 0) devices[0] = c->device;
    return c->device == FTS_DEVICE_NONE ? 0 : 1;
  }
  for (int j = 0; j < (int)c->shards.size() && j < cap; j++)
    if (devices) devices[j] = c->shards[j]->device;
  return (int)c->shards.size();
}

}  // extern "C"

static int multi_rp_verify(fts_ctx* c, size_t n, const uint8_t* const* der, const size_t* len, const uint8_t* com64,
                           int32_t* status) {
  return run_shards(plan(n, nullptr, (int)c->shards.size()), [&](int j, size_t lo, size_t hi) {
    return fts_rp_verify_batch(c->shards[j], hi - lo, der + lo, len + lo, com64 + 64 * lo, status + lo);
  });
}

// cost weight of an action: its range proofs (none for a 1-in/1-out transfer) + the sigma proof
static double action_weight(size_t n_in, size_t n_out, bool transfer) {
  return (transfer && n_in == 1 && n_out == 1 ? 0.0 : (double)n_out) + 0.25;
}

extern "C" {

int fts_ctx_create(const uint8_t* pp, size_t pp_len, int device, fts_ctx** out) {
  return ctx_create(pp, pp_len, 0, device, out);
}
int fts_ctx_create_opts(const uint8_t* pp, size_t pp_len, int device, const fts_ctx_opts* opts, fts_ctx** out) {
  return ctx_create(pp, pp_len, opts ? opts->bit_length : 0, device, out, opts);
}
int fts_ctx_create_bits(const uint8_t* pp, size_t pp_len, uint32_t bit_length, int device, fts_ctx** out) {
  return ctx_create(pp, pp_len, bit_length, device, out);
}

void fts_ctx_destroy(fts_ctx* c) {
  if (!c) return;
  for (fts_ctx* ch : c->shards) fts_ctx_destroy(ch);
  c->shards.clear();
  if (c->device == FTS_DEVICE_NONE || c->lanes.empty()) {
    delete c;
    return;
  }
  hipSetDevice(c->device);
  for (Lane* L : c->lanes) {
    if (L->s) hipStreamSynchronize(L->s);
    if (L->s2 && L->s2 != L->s) hipStreamSynchronize(L->s2);
    if (L->s4 && L->s4 != L->s) hipStreamSynchronize(L->s4);
    if (L->s3) hipStreamSynchronize(L->s3);
    L->ws.release();
    if (L->s3) hipStreamDestroy(L->s3);
    if (L->ev_a) hipEventDestroy(L->ev_a);
    if (L->ev_b) hipEventDestroy(L->ev_b);
    if (L->ev_c) hipEventDestroy(L->ev_c);
    if (L->ev_d) hipEventDestroy(L->ev_d);
    if (L->ev_e) hipEventDestroy(L->ev_e);
    L->tl.destroy();
    if (L->done) hipEventDestroy(L->done);
    if (L->s2 && L->s2 != L->s) hipStreamDestroy(L->s2);
    if (L->s4 && L->s4 != L->s) hipStreamDestroy(L->s4);
    if (L->s) hipStreamDestroy(L->s);
    L->free_pinned();
    delete L;
  }
  if (c->d_tables) hipFree(c->d_tables);
  if (c->d_wtables) hipFree(c->d_wtables);
  if (c->d_x0const) hipFree(c->d_x0const);
  if (c->d_x0tmpl) hipFree(c->d_x0tmpl);
  for (RpSlot* sl : c->slots) {
    if (sl->s) hipStreamSynchronize(sl->s);
    if (sl->dev) hipFree(sl->dev);
    if (sl->pin) (void)hipHostFree(sl->pin);
    if (sl->done) hipEventDestroy(sl->done);
    if (sl->s) hipStreamDestroy(sl->s);
    delete sl->b;
    delete sl;
  }
  for (ActSlot* sl : c->aslots) {
    if (sl->s) hipStreamSynchronize(sl->s);
    if (sl->dev) hipFree(sl->dev);
    if (sl->pin) (void)hipHostFree(sl->pin);
    if (sl->done) hipEventDestroy(sl->done);
    for (hipEvent_t e : sl->ev_sig)
      if (e) hipEventDestroy(e);
    if (sl->s) hipStreamDestroy(sl->s);
    delete sl->b;
    delete sl;
  }
  delete c;
}

int fts_ctx_info(const fts_ctx* c, fts_pp_info* o) {
  if (!c || !o) return FTS_API_EINVAL;
  if (!c->shards.empty()) {  // device of shard 0; tables summed over the devices
    int rc = fts_ctx_info(c->shards[0], o);
    for (size_t j = 1; j < c->shards.size(); j++) o->table_bytes += c->shards[j]->table_bytes;
    return rc;
  }
  o->bit_length = (uint32_t)c->pp.bit_length;
  o->rounds = (uint32_t)c->pp.rounds;
  o->curve_id = (uint32_t)c->pp.curve_id;
  o->device = c->device;
  o->max_token = c->pp.max_token;
  o->table_bytes = c->table_bytes;
  o->wide_bits = (uint32_t)c->wbits;
  o->lanes = (uint32_t)c->nlanes;
  return FTS_API_OK;
}

const char* fts_status_str(int32_t s) {
  switch (s) {
    case FTS_OK: return "";
    case FTS_E_MALFORMED: return "failed to deserialize proof";
    case FTS_E_RP_NIL: return "invalid range proof: nil elements";
    case FTS_E_RP_INVALID: return "invalid range proof";
    case FTS_E_IPA_NIL: return "invalid IPA proof: nil elements";
    case FTS_E_IPA_LEN: return "invalid IPA proof";
    case FTS_E_IPA_INVALID: return "invalid IPA";
    case FTS_E_RC_COUNT: return "invalid range proof";
    case FTS_E_TAS_INVALID: return "invalid sum and type proof";
    case FTS_E_ST_INVALID: return "invalid same type proof";
    case FTS_E_NOT_RUN: return "not evaluated";
    case FTS_E_ACTION_INVALID: return "invalid action";
    case FTS_E_OPEN_MISMATCH: return "does not match the provided opening";
    case FTS_E_SIG_MALFORMED: return "asn1: signature does not deserialize";
    case FTS_E_SIG_NOT_LOW_S: return "signature is not in lowS";
    case FTS_E_SIG_INVALID: return "signature not valid";
    case FTS_E_NYM_MALFORMED: return "error unmarshalling signature";
    case FTS_E_NYM_BADKEY: return "failed importing nym public key";
    case FTS_E_NYM_INVALID: return "pseudonym signature invalid: zero-knowledge proof is invalid";
    case FTS_E_ID_MALFORMED: return "identity malformed";
    case FTS_E_ID_BADNYM: return "failed to import nym public key";
    case FTS_E_ID_NO_EIDNYM: return "no EidNym provided but ExpectEidNym required";
    case FTS_E_ID_NO_RHNYM: return "no RhNym provided but ExpectEidNymRhNym required";
    case FTS_E_ID_REVOCATION: return "unsupported revocation algorithm";
    case FTS_E_ID_APRIME: return "signature invalid: APrime = 1";
    case FTS_E_ID_PAIRING: return "signature invalid: APrime and ABar don't have the expected structure";
    case FTS_E_ID_ZK: return "signature invalid: zero-knowledge proof is invalid";
    default: return "unknown status";
  }
}

int fts_last_timings(const fts_ctx* c, const char** names, float* ms, int cap) {
  return fts_last_timings_ex(c, names, ms, nullptr, cap);
}

int fts_last_timings_ex(const fts_ctx* cc, const char** names, float* ms, double* mads, int cap) {
  if (!cc) return 0;
  if (!cc->shards.empty()) return fts_last_timings_ex(cc->shards[0], names, ms, mads, cap);
  fts_ctx* c = const_cast<fts_ctx*>(cc);
  std::lock_guard<std::mutex> g(c->tim_mu);
  int m = std::min(cap, c->ntim);
  for (int i = 0; i < m; i++) {
    if (names) names[i] = c->tim_name[i];
    if (ms) ms[i] = c->tim_ms[i];
    if (mads) mads[i] = c->tim_work[i] * MADS_PER_MUL;
  }
  return m;
}

}  // extern "C"

// ------------------------------------------------------------ range proofs
// host records for B proofs
struct RpHost {
  std::vector<uint8_t> raw;
  std::vector<uint32_t> sc;
  std::vector<int32_t> status, ipa;
};

// DER range proofs -> device input records (raw BE points with the caller's
// commitment in slot V, canonical scalars, host-parse verdicts), written into
// caller-provided host memory (pageable or pinned); parallel over chunks of
// 256 proofs on the host pool
static void parse_rp_into(int k, size_t B, const uint8_t* const* der_p, const size_t* der_len, const uint8_t* com64,
                          uint8_t* raw, uint32_t* sc, int32_t* status, int32_t* ipa) {
  const int npts = rp_npts(k);
  constexpr size_t CH = 256;
  parallel_for((B + CH - 1) / CH, 2, [&](size_t c) {
    for (size_t i = c * CH; i < std::min(B, (c + 1) * CH); i++) {
      uint8_t* pts = raw + i * npts * 64;  // every slot written once below (no clearing pass)
      status[i] = 0;
      ipa[i] = 0;
      der::Span s{der_p[i], der_len[i]};
      if (!der_p[i]) s.n = 0;
      parse_range_proof(s, k, pts, sc + i * RP_NSC * 8, status[i], ipa[i]);
      memcpy(pts + RP_PT_V * 64, com64 + i * 64, 64);
    }
  });
}

static void parse_rp_batch(int k, size_t B, const uint8_t* const* der_p, const size_t* der_len, const uint8_t* com64,
                           RpHost& h) {
  const int npts = rp_npts(k);
  h.raw.assign(B * npts * 64, 0);
  h.sc.assign(B * RP_NSC * 8, 0);
  h.status.assign(B, 0);
  h.ipa.assign(B, 0);
  parse_rp_into(k, B, der_p, der_len, com64, h.raw.data(), h.sc.data(), h.status.data(), h.ipa.data());
}

// sig_ms (optional): the k_sig_prep / k_sig_finish spans of an action call's slot
static void collect_timings(fts_ctx* c, Lane& L, fts_rp_batch* b, const float* sig_ms = nullptr) {
  std::lock_guard<std::mutex> g(c->tim_mu);
  c->ntim = 0;
  c->last_lane = L.id;
  for (int q = 0; sig_ms && q < 2; q++) {
    c->tim_name[c->ntim] = q ? "k_sig_finish" : "k_sig_prep";
    c->tim_ms[c->ntim] = sig_ms[q];
    c->tim_work[c->ntim++] = 0;
  }
  for (int i = 0; i < L.tl.n && c->ntim < Timeline::CAP; i++) {
    if (!L.tl.name[i]) continue;  // fork/join markers
    const int j = c->ntim++;
    c->tim_name[j] = L.tl.name[i];
    c->tim_work[j] = L.tl.work[i];
    hipEventElapsedTime(&c->tim_ms[j], L.tl.ev[L.tl.start[i]], L.tl.ev[i + 1]);
  }
  const char* hn[8] = {"host_prep", "host_enqueue", "host_wait_flag", "host_parse", "host_stage", "host_misc",
                       "host_total", "host_stage_copy"};
  const float hv[8] = {L.host_prep_ms, L.host_enqueue_ms, L.host_wait_ms, L.host_parse_ms, L.host_stage_ms,
                       L.host_misc_ms, L.host_total_ms, L.host_stage_copy_ms};
  for (int q = 0; q < 8 && c->ntim < Timeline::CAP; q++) {
    c->tim_name[c->ntim] = hn[q];
    c->tim_ms[c->ntim] = hv[q];
    c->tim_work[c->ntim] = 0;
    c->ntim++;
  }
  if (b) {
    b->ntim = c->ntim;
    for (int j = 0; j < c->ntim; j++) {
      b->tim_name[j] = c->tim_name[j];
      b->tim_ms[j] = c->tim_ms[j];
      b->tim_work[j] = c->tim_work[j];
    }
  }
}

// MSM plan for N real points on lane L's workspace (buffers grown as needed,
// window table uploaded on L.s).  Returns 0 or FTS_API_ENOMEM.
static int msm_prepare_plan(Lane& L, MsmPlan& mp, int slot);
static int msm_prepare(Lane& L, int N, MsmPlan& mp, int slot, int ch, bool local_sort, int maxc) {
  mp = MsmPlan{};
  msm_layout(N, mp, maxc);
  if (ch != MSM_CH) msm_set_chunk(mp, ch);
  mp.local_sort = local_sort;
  return msm_prepare_plan(L, mp, slot);
}
// buffers of an already laid-out plan (msm_layout / msm_layout_groups) on lane L.
// `slot` (< MSM_WIN_SLOTS) is the pinned source of the window-table upload: plans
// uploaded before the lane's next sync must use different slots (MSM_SLOT_*)
static int msm_prepare_plan(Lane& L, MsmPlan& mp, int slot) {
  Workspace& w = L.ws;
  if (w.m_choff.ensure((size_t)mp.NB * 4) || w.m_chbkt.ensure((size_t)mp.NC * 4) ||
      w.m_partials.ensure((size_t)mp.NC * 96) || w.m_keys.ensure((size_t)mp.nw * mp.NV * 4) ||
      w.m_counts.ensure((size_t)mp.NB * 4) || w.m_offsets.ensure((size_t)mp.NB * 4) ||
      w.m_cursor.ensure((size_t)mp.nw * mp.NV * 4) || w.m_sorted.ensure((size_t)mp.nw * mp.NV * 4) ||
      w.m_buckets.ensure((size_t)mp.NB * 96) || w.m_segs.ensure((size_t)mp.NS * 96) ||
      w.m_wins.ensure((size_t)(mp.nw + 1) * 96) || w.m_out.ensure((size_t)mp.G * 96) ||
      w.m_scratch.ensure(std::max((size_t)mp.NS * 96, msm_scratch_words(mp) * 4)) || w.m_win.ensure(sizeof(mp.win)))
    return FTS_API_ENOMEM;
  mp.d_win = w.m_win.as<MsmWindow>();
  MsmWindow* src = L.pin->win[slot];
  memcpy(src, mp.win, sizeof(MsmWindow) * mp.nw);
  if (hipMemcpyAsync(mp.d_win, src, sizeof(MsmWindow) * mp.nw, hipMemcpyHostToDevice, L.s) != hipSuccess)
    return FTS_API_EDEVICE;
  mp.keys = w.m_keys.as<int32_t>();
  mp.counts = w.m_counts.as<uint32_t>();
  mp.offsets = w.m_offsets.as<uint32_t>();
  mp.cursor = w.m_cursor.as<uint32_t>();
  mp.sorted = w.m_sorted.as<uint32_t>();
  mp.buckets = w.m_buckets.as<uint32_t>();
  mp.segs = w.m_segs.as<uint32_t>();
  mp.wins = w.m_wins.as<uint32_t>();
  mp.out = w.m_out.as<uint32_t>();
  mp.chunk_off = w.m_choff.as<uint32_t>();
  mp.chunk_bkt = w.m_chbkt.as<int32_t>();
  mp.partials = w.m_partials.as<uint32_t>();
  mp.scratch = w.m_scratch.as<uint32_t>();
  return FTS_API_OK;
}

// workspace of a range-proof pass of B proofs (grow-only).  The pass's INPUT
// buffers (w.rp_* for gathered/action batches) belong to the caller, which
// fills them before rp_pipeline runs: they are never re-allocated here.
static int rp_buffers(fts_ctx* c, Lane& L, int B) {
  const int n = c->n, k = c->k, npts = rp_npts(k), N = B * npts;
  Workspace& w = L.ws;
  if (w.pts.ensure((size_t)B * npts * 64) || w.ch.ensure((size_t)B * rp_nch(k) * 32) ||
      w.small.ensure((size_t)B * (2 + k) * SMALL_SLOT) || w.hpj.ensure((size_t)B * (n + 1) * 96) ||
      w.hpa.ensure((size_t)B * (n + 1) * 64) || w.hpbe.ensure((size_t)B * (n + 1) * 64) ||
      w.x0.ensure((size_t)B * x0_var_bytes(n)) || w.x0mid.ensure((size_t)B * 32) || w.terms.ensure(rp_terms_words(B, n, k) * 4) ||
      w.scratch.ensure(std::max(rp_scratch_words(B, n, k), (size_t)B * 10 * 24) * 4) || w.r_key.ensure(32) ||
      w.r_msc.ensure((size_t)N * 32) || w.r_coef.ensure((size_t)B * RLC_NCOEF * 32) ||
      w.r_colsum.ensure(rlc_ncols(n) * 32 * (1 + 64))  /* + RQ_PARTS partial rows of column Q */ || w.r_fixed.ensure(rlc_ncols(n) * 96) || w.r_flag.ensure(4) || w.ypow.ensure((size_t)B * n * 32) ||
      w.svec.ensure((size_t)B * n * 32) || w.zvec.ensure((size_t)B * n * 32) || w.rp_excl.ensure((size_t)B * 4) ||
      !L.status_buf((size_t)B))
    return FTS_API_ENOMEM;
  return FTS_API_OK;
}

// size lane L's workspace for range-proof passes of up to B proofs; with
// inputs, also the pass-input buffers (w.rp_*) -- never from inside a pass,
// whose caller has already filled them
static int lane_reserve(fts_ctx* c, Lane& L, int B, bool inputs) {
  const int npts = rp_npts(c->k);
  MsmPlan big{};
  if (int rc = msm_prepare(L, B * npts, big, MSM_SLOT_RESERVE, MSM_CH, c->msm_sort != 0, c->msm_maxc)) return rc;
  if (int rc = rp_buffers(c, L, B)) return rc;
  Workspace& w = L.ws;
  if (inputs && (w.rp_raw.ensure((size_t)B * npts * 64) || w.rp_sc.ensure((size_t)B * RP_NSC * 32) ||
                 w.rp_status.ensure((size_t)B * 4) || w.rp_ipa.ensure((size_t)B * 4)))
    return FTS_API_ENOMEM;
  L.presized = true;
  return FTS_API_OK;
}

// The batch check failed: find the failing proofs without re-checking the whole
// pass proof by proof ("fall back to per-proof checks
// (bisection)").  Round 1 tests groups of RP_GT1 consecutive proofs that never
// straddle two caller batches (`groups`: the batches' first proofs, the pass's
// end last); if more than RP_GT2_MIN proofs sit in failing groups, round 2 tests
// groups of RP_GT2 among them.  Every group test is ONE grouped MSM over the
// batch check's own weights.  The proofs of groups that do not close get the
// per-proof final equations (bulletproof.go:314-324, ipa.go:254-259), whose
// verdicts are the reference's.  A single bad proof costs one grouped MSM plus
// RP_GT1 per-proof checks, all of them in its own caller batch (RP_GT1, RP_GT2_MIN:
// fts_ctx::gt1, gt2_min).
constexpr int RP_GT2 = 8;
// dense[q] (caller batch q = [groups[q], groups[q+1])): its round-1 groups are of
// RP_GT2 proofs instead of gt1; with FTS_GT_ADAPT the flags are updated from this
// fallback's round-1 failures (a batch's own density).  An empty `dense` = all sparse.
// only (optional): only[q] != 0 for the caller batches whose own combination failed
// (the per-caller-batch main check): the others are decided and stay out of it
static int rp_group_fallback(fts_ctx* c, Lane& L, const RpBatchDev& d, const RlcDev& r,
                             const std::vector<int>& groups, std::vector<uint8_t>& dense,
                             const std::vector<uint8_t>* only = nullptr) {
  const bool adapt = c->gt_adapt && c->gt1 > RP_GT2;
  const int RP_GT2_MIN = c->gt2_min;
  const int B = d.B, n = d.n, npts = rp_npts(d.k);
  const size_t nb = groups.size() > 0 ? groups.size() - 1 : 0;
  dense.resize(nb, 0);
  Workspace& w = L.ws;
  L.tl.fallback();
  // round-1 selections, -1 padded: groups of gt1 over the sparse batches, of RP_GT2 over the dense ones
  std::vector<int32_t> sel_big, sel_small;
  for (size_t q = 0; q < nb; q++) {
    if (only && !(*only)[q]) continue;
    const bool small = adapt && dense[q];
    const int gs = small ? RP_GT2 : c->gt1;
    std::vector<int32_t>& sel = small ? sel_small : sel_big;
    for (int lo = groups[q]; lo < groups[q + 1]; lo += gs)
      for (int j = 0; j < gs; j++) sel.push_back(lo + j < groups[q + 1] ? lo + j : -1);
  }
  const size_t slots = std::max<size_t>(sel_big.size() + sel_small.size(), (size_t)B + RP_GT2);
  // groups of any round: round 1 has sel_big / gt1 + sel_small / RP_GT2, round 2 at most slots / RP_GT2
  const size_t gmax = std::max(sel_big.size() / c->gt1 + sel_small.size() / RP_GT2, (slots + RP_GT2 - 1) / RP_GT2);
  if (w.r_sel.ensure(2 * slots * 4) || w.r_next.ensure(slots * 4) || w.r_cnt.ensure(8) ||
      w.r_gcol.ensure(gmax * rlc_ncols(n) * 32) || w.r_gfix.ensure(gmax * rlc_ncols(n) * 96))
    return FTS_API_ENOMEM;
  uint8_t* hs = L.stage_buf((sel_big.size() + sel_small.size()) * 4);
  if (!hs) return FTS_API_ENOMEM;
  memcpy(hs, sel_big.data(), sel_big.size() * 4);
  memcpy(hs + sel_big.size() * 4, sel_small.data(), sel_small.size() * 4);
  int32_t* cur_big = w.r_sel.as<int32_t>();
  int32_t* cur_small = cur_big + sel_big.size();
  int32_t* nxt = w.r_next.as<int32_t>();
  uint32_t* cnt = w.r_cnt.as<uint32_t>();
  HIP_OK(hipMemcpyAsync(cur_big, hs, (sel_big.size() + sel_small.size()) * 4, hipMemcpyHostToDevice, L.s));
  HIP_OK(hipMemsetAsync(nxt, 0xff, slots * 4, L.s));  // -1: empty slots of the next round
  HIP_OK(hipMemsetAsync(cnt, 0, 4, L.s));
  // one grouped test per group size; both append their failing proofs to nxt
  auto group_test = [&](const int32_t* sel, int G, int gs) -> int {
    if (G == 0) return FTS_API_OK;
    MsmPlan gp{};
    msm_layout_groups(G * gs * npts, G, gs * npts, gp, c->msm_maxc);
    gp.local_sort = c->msm_sort != 0;  // FTS_MSM_SORT covers the group tests' MSMs too
    gp.sel = sel;
    gp.sel_pts = npts;
    if (int rc = msm_prepare_plan(L, gp, gs == RP_GT2 ? MSM_SLOT_GT_SMALL : MSM_SLOT_GT_BIG)) return rc;
    launch_rlc_group_test(d, r, c->d_tables, gp, sel, G, gs, w.r_gcol.as<uint32_t>(), w.r_gfix.as<uint32_t>(), nxt,
                          cnt, L.s, &L.tl);
    HIP_OK(hipGetLastError());
    return FTS_API_OK;
  };
  if (int rc = group_test(cur_big, (int)(sel_big.size() / c->gt1), c->gt1)) return rc;
  if (int rc = group_test(cur_small, (int)(sel_small.size() / RP_GT2), RP_GT2)) return rc;
  HIP_OK(hipMemcpyAsync(&L.pin->flag, cnt, 4, hipMemcpyDeviceToHost, L.s));
  HIP_OK(L.sync());
  const int nfail = L.pin->flag;
  if (adapt && nfail > 0) {
    // each batch's own density from its failing round-1 proofs
    int32_t* hf = L.status_buf((size_t)nfail);
    if (!hf) return FTS_API_ENOMEM;
    HIP_OK(hipMemcpyAsync(hf, nxt, (size_t)nfail * 4, hipMemcpyDeviceToHost, L.s));
    HIP_OK(L.sync());
    std::vector<int> fails(nb, 0);
    for (int i = 0; i < nfail; i++) {
      const size_t q = (size_t)(std::upper_bound(groups.begin(), groups.end(), hf[i]) - groups.begin()) - 1;
      if (q < nb) fails[q]++;
    }
    for (size_t q = 0; q < nb; q++) {
      const int sz = groups[q + 1] - groups[q];
      if (only && !(*only)[q]) dense[q] = 0;  // its combination closed: no bad proof
      else dense[q] = dense[q] ? fails[q] > 0.02 * sz : fails[q] > 0.5 * sz;
    }
  } else if (adapt) {
    std::fill(dense.begin(), dense.end(), 0);
  }
  if (nfail == 0) return FTS_API_OK;
  // per-proof checks of what is left; a second group test only pays when round 1
  // left many proofs in large groups (the per-proof check's latency is one GLV
  // chain whatever their number, its work grows with it)
  if (sel_big.empty() || nfail <= RP_GT2_MIN) {
    launch_rp_fallback(d, c->d_tables, nxt, nfail, L.s, &L.tl);
    HIP_OK(hipGetLastError());
    return FTS_API_OK;
  }
  int32_t* cur = w.r_sel.as<int32_t>();  // round 2 over the survivors, groups of RP_GT2
  HIP_OK(hipMemcpyAsync(cur, nxt, slots * 4, hipMemcpyDeviceToDevice, L.s));
  HIP_OK(hipMemsetAsync(nxt, 0xff, slots * 4, L.s));
  HIP_OK(hipMemsetAsync(cnt, 0, 4, L.s));
  const int G2 = (nfail + RP_GT2 - 1) / RP_GT2;
  if ((size_t)G2 > gmax) return FTS_API_EINVAL;  // cannot happen: nfail <= B
  if (int rc = group_test(cur, G2, RP_GT2)) return rc;
  HIP_OK(hipMemcpyAsync(&L.pin->flag, cnt, 4, hipMemcpyDeviceToHost, L.s));
  HIP_OK(L.sync());
  const int nfail2 = L.pin->flag;
  if (nfail2 == 0) return FTS_API_OK;
  launch_rp_fallback(d, c->d_tables, nxt, nfail2, L.s, &L.tl);
  HIP_OK(hipGetLastError());
  return FTS_API_OK;
}

// One range-proof pass enqueued on a lane (rp_enqueue), finished by rp_finish.
struct RpPass {
  RpBatchDev d{};
  RlcDev r{};
  std::vector<int> groups;
  std::vector<uint8_t> dense;  // per caller batch (groups[q] .. groups[q+1]): round-1 groups of 8; updated by the fallback
  double t_start = 0, t_prep = 0, t_enq = 0;
  bool tl_started = false;
  std::vector<fts_rp_batch*> bats;  // the caller batches of the pass (groups order); empty: none
  bool clean = false;               // the combination closed: no fallback ran (rp_finish)
  int located = -1;                 // the locator: 1 hit, 0 missed, -1 not run  // the lane's timeline was begun by the caller (action passes: gather + sigma marks)
};

// Range-proof pipeline on B proofs already on the device: exact phase, RLC
// batch check, and (rp_finish) the group-test fallback when the combination
// fails.  `between` (optional) is launched after the RLC check and before the
// flag sync (the sigma-proof kernels of transfer/issue batches).
// `groups`: first proof of every caller batch in the pass, then B ({0, B}: one batch)
// `pre_rlc` (optional): launched on the batch check's stream (lane s3) right before k_rlc_prep
template <class F>
static int rp_enqueue(fts_ctx* c, Lane& L, int B, uint8_t* d_raw, uint32_t* d_sc, int32_t* d_status, int32_t* d_ipa,
                      F&& between, const std::vector<int>& groups, RpPass& P,
                      void (*pre_rlc)(void*, hipStream_t) = nullptr, void* pre_rlc_arg = nullptr) {
  const int n = c->n, k = c->k, npts = rp_npts(k);
  Workspace& w = L.ws;
  const int N = B * npts;
  P.t_start = now_ms();
  P.groups = groups;
  // first range-proof pass of this lane: size the workspace for the largest
  // coalesced pass at once (no re-allocation, i.e. no device-wide sync, later)
  if (!L.presized && c->coalesce_max > (size_t)B && c->coalesce_max <= (1u << 20))
    if (int rc = lane_reserve(c, L, (int)c->coalesce_max, false)) return rc;
  MsmPlan mp{};
  // the per-caller-batch combination: G groups of gs proof slots (padding -1)
  const int G = (int)groups.size() - 1;
  const bool grouped = c->main_groups && G > 1 && G <= RP_GATHER_MAX && !pre_rlc;
  int gs = 0;
  if (grouped) {
    for (int q = 0; q < G; q++) gs = std::max(gs, groups[q + 1] - groups[q]);
    msm_layout_groups(G * gs * npts, G, gs * npts, mp, c->msm_maxc);
    mp.local_sort = c->msm_sort != 0;
    Workspace& w0 = L.ws;
    const size_t NC = rlc_ncols(n);
    if (w0.r_msel.ensure((size_t)G * gs * 4) || w0.r_mcol.ensure((size_t)G * NC * 32) ||
        w0.r_mfix.ensure((size_t)G * NC * 96) || w0.r_mqfix.ensure((size_t)G * NC * 96) ||
        w0.r_mflag.ensure((size_t)G * 4))
      return FTS_API_ENOMEM;
    int32_t* hs = L.sel_buf((size_t)G * gs);
    if (!hs) return FTS_API_ENOMEM;
    for (int q = 0; q < G; q++)
      for (int j = 0; j < gs; j++) hs[(size_t)q * gs + j] = groups[q] + j < groups[q + 1] ? groups[q] + j : -1;
    HIP_OK(hipMemcpyAsync(w0.r_msel.p, hs, (size_t)G * gs * 4, hipMemcpyHostToDevice, L.s));
    // equal caller batches (the usual coalesced pass): slot = proof, no indirection in
    // the MSM's point gathers
    bool uniform = true;
    for (int q = 0; q < G; q++) uniform = uniform && groups[q] == q * gs;
    mp.sel = uniform && groups[G] == G * gs ? nullptr : w0.r_msel.as<int32_t>();
    mp.sel_pts = npts;
    if (int rc = msm_prepare_plan(L, mp, MSM_SLOT_PASS)) return rc;
  } else if (int rc = msm_prepare(L, N, mp, MSM_SLOT_PASS, MSM_CH, c->msm_sort != 0, c->msm_maxc)) {
    return rc;
  }
  if (int rc = rp_buffers(c, L, B)) return rc;
  RpBatchDev d{B,
               n,
               k,
               d_raw,
               d_sc,
               d_status,
               d_ipa,
               w.pts.as<uint32_t>(),
               w.ch.as<uint32_t>(),
               w.small.as<uint8_t>(),
               w.hpj.as<uint32_t>(),
               w.hpa.as<uint32_t>(),
               w.hpbe.as<uint8_t>(),
               w.x0.as<uint8_t>(),
               w.terms.as<uint32_t>(),
               w.scratch.as<uint32_t>(),
               w.ypow.as<uint32_t>(),
               w.svec.as<uint32_t>(),
               w.zvec.as<uint32_t>(),
               nullptr,
               nullptr,
               (size_t)B <= c->com_fixed_max && L.alone ? 1 : 0};
  d.pre_rlc = pre_rlc;
  d.pre_rlc_arg = pre_rlc_arg;
  // 2 (adaptive): 0 on the latency path, 1 on the work path; 3: 0 on the latency
  // path, on the work path the MSM's sort beside the fixed-base launch
  d.rlc_fork = c->rlc_fork == 2 ? (d.com_fixed ? 0 : 1) : c->rlc_fork >= 3 ? (d.com_fixed ? 0 : c->rlc_fork) : c->rlc_fork;
  d.ev_coef = L.ev_c;
  d.ev_fx = L.ev_d;
  // x0 prefix beside the com chain (work path) or com_tree (latency path; round 2
  // measured that slower, 3.51 vs 3.06 ms, when the normalisation did not yet write
  // the H' records and the prefix waited for a separate build)
  d.x0_mid = (c->x0_split & (d.com_fixed ? 2 : 1)) ? w.x0mid.as<uint32_t>() : nullptr;
  d.excl = pre_rlc ? w.rp_excl.as<int32_t>() : nullptr;
  RlcDev r{w.r_key.as<uint32_t>(), w.r_msc.as<uint32_t>(),   w.r_coef.as<uint32_t>(), w.r_colsum.as<uint32_t>(),
           w.r_fixed.as<uint32_t>(), w.r_flag.as<int32_t>(), w.m_scratch.as<uint32_t>(), mp};
  if (grouped) {
    r.G = G;
    r.gs = gs;
    r.sel = w.r_msel.as<int32_t>();
    r.gcol = w.r_mcol.as<uint32_t>();
    r.gfix = w.r_mfix.as<uint32_t>();
    r.gqfix = w.r_mqfix.as<uint32_t>();
    r.gflag = w.r_mflag.as<int32_t>();
  }
  // fresh RLC weights key (getrandom), unpredictable to the provers
  if (getrandom(L.pin->key, sizeof L.pin->key, 0) != (ssize_t)sizeof L.pin->key) return FTS_API_EDEVICE;
  HIP_OK(hipMemcpyAsync(r.key, L.pin->key, sizeof L.pin->key, hipMemcpyHostToDevice, L.s));
  P.t_prep = now_ms();
  if (!P.tl_started) L.tl.begin(L.s);
  if (c->fx_serial) {
    // the wait, this pass's fixed-base launch and its event record are enqueued in
    // one critical section, so the chain of events follows the enqueue order
    std::lock_guard<std::mutex> g(c->fx_mu);
    d.fx_wait = c->fx_last;
    launch_rp_batch(d, r, c->d_tables, c->d_wtables, c->d_x0const, c->d_x0tmpl, L.s, L.s2, L.s3, L.s4, &L.tl,
                    c->wbits);
    c->fx_last = d.ev_fx;
  } else {
    launch_rp_batch(d, r, c->d_tables, c->d_wtables, c->d_x0const, c->d_x0tmpl, L.s, L.s2, L.s3, L.s4, &L.tl,
                    c->wbits);
  }
  between();
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(&L.pin->flag, r.flag, 4, hipMemcpyDeviceToHost, L.s));
  if (grouped) HIP_OK(hipMemcpyAsync(L.pin->gflag, r.gflag, (size_t)G * 4, hipMemcpyDeviceToHost, L.s));
  P.t_enq = now_ms();
  P.d = d;
  P.r = r;
  return FTS_API_OK;
}

// The single-fault locator (rp_kernels.hip k_rlc_locate): S' = (j + 1) S locates
// the one bad proof j of a failed combination S.  Its per-proof final equations
// give its verdict (bulletproof.go:314-324, ipa.go:254-259), and every other proof
// is accepted -- the combination of the others is S - rho_j E_j = 0 with the
// batch check's own soundness.  -> 1 decided, 0 not a single fault (the group test
// decides), < 0 an API error.  The workspace's weights are index-weighted after it,
// which the group test accepts as its weights (any fresh random weights do).
static int rp_locate_single(fts_ctx* c, Lane& L, RpPass& P) {
  const int B = P.d.B;
  Workspace& w = L.ws;
  if (w.r_loc.ensure(4) || w.r_save.ensure(96)) return FTS_API_ENOMEM;
  L.tl.fallback();
  int32_t* loc = w.r_loc.as<int32_t>();
  HIP_OK(hipMemsetAsync(loc, 0xff, 4, L.s));
  launch_rlc_locate(P.d, P.r, c->d_tables, w.r_save.as<uint32_t>(), loc, L.s, &L.tl);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(&L.pin->flag, loc, 4, hipMemcpyDeviceToHost, L.s));
  HIP_OK(L.sync());
  const int i = L.pin->flag;
  if (i < 0 || i >= B) return 0;
  launch_rp_fallback(P.d, c->d_tables, loc, 1, L.s, &L.tl);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(&L.pin->flag, P.d.status + i, 4, hipMemcpyDeviceToHost, L.s));
  HIP_OK(L.sync());
  if (L.pin->flag == FTS_OK) return 0;  // not a fault after all: the group test decides
  launch_rlc_accept_except(B, i, P.d.status, P.d.ipa_flag, L.s);
  HIP_OK(hipGetLastError());
  std::fill(P.dense.begin(), P.dense.end(), 0);
  return 1;
}

// wait for an enqueued pass; on a failed combination, the single-fault locator,
// then (several bad proofs) the group-test fallback
static int rp_finish(fts_ctx* c, Lane& L, RpPass& P) {
  HIP_OK(L.sync());
  const double t_wait = now_ms();
  L.host_prep_ms = (float)(P.t_prep - P.t_start);
  L.host_enqueue_ms = (float)(P.t_enq - P.t_prep);
  L.host_wait_ms = (float)(t_wait - P.t_enq);
  const int32_t flag = L.pin->flag;
  c->last_fallback = flag ? 0 : 1;
  P.clean = flag != 0;
  if (flag) return FTS_API_OK;
  if (P.r.G > 1) {  // per-caller-batch combination: only the failing batches go to the group test
    std::vector<uint8_t> only((size_t)P.r.G, 0);
    for (int q = 0; q < P.r.G; q++) only[q] = L.pin->gflag[q] ? 0 : 1;
    return rp_group_fallback(c, L, P.d, P.r, P.groups, P.dense, &only);
  }
  if (c->locate && P.d.B > 1 && std::none_of(P.dense.begin(), P.dense.end(), [](uint8_t x) { return x != 0; })) {
    // a batch of the pass still in its backoff skips the locator for the whole pass
    bool skip = false;
    for (fts_rp_batch* b : P.bats)
      if (b->locate_skip > 0) {
        b->locate_skip--;
        skip = true;
      }
    if (!skip) {
      const int rc = rp_locate_single(c, L, P);
      if (rc < 0) return rc;
      P.located = rc;
      if (rc == 1) {
        for (fts_rp_batch* b : P.bats) b->locate_backoff = 8;
        return FTS_API_OK;
      }
      // missed: the batches holding bad proofs back off once the verdicts are in (run_rp_groups)
    }
  }
  return rp_group_fallback(c, L, P.d, P.r, P.groups, P.dense);
}

template <class F>
static int rp_pipeline(fts_ctx* c, Lane& L, int B, uint8_t* d_raw, uint32_t* d_sc, int32_t* d_status, int32_t* d_ipa,
                       F&& between, const std::vector<int>& groups, void (*pre_rlc)(void*, hipStream_t) = nullptr,
                       void* pre_rlc_arg = nullptr) {
  RpPass P;
  if (int rc = rp_enqueue(c, L, B, d_raw, d_sc, d_status, d_ipa, between, groups, P, pre_rlc, pre_rlc_arg)) return rc;
  return rp_finish(c, L, P);
}

// Device passes over groups of staged batches, group j on lanes[j] (the
// dispatcher passes one group; several are enqueued back to back before any is
// waited for): a single batch runs in place; several are gathered (D2D) into the
// lane's contiguous input buffers, verified as one batch, and their verdicts
// scattered back.  rc[j] is the status of group j's requests.  (Round 4 measured
// staggered sub-passes of one coalesced group -- sub-pass j's fixed-base launch
// after sub-pass j-1's -- and dropped them: 20-batch bursts 3.77-3.89 vs 3.95-3.97
// M rp64/s as one pass)
// the pre_rlc hook of a pass with action calls: wait for their sigma equations, then
// exclude the range proofs of actions whose sigma proof failed (pass offsets `off`)
struct SigHook {
  Lane* L = nullptr;
  std::vector<const SigBatchDev*> sig;
  std::vector<int> off;  // first range proof of the call in the pass (-1: none)
  std::vector<hipEvent_t> ev;  // the call's sigma-done event (its slot's ev_sig[2])
};

static void run_rp_groups(fts_ctx* c, const std::vector<Lane*>& lanes, const std::vector<std::vector<RpReq*>>& sub,
                             std::vector<int>& rc) {
  const size_t m = sub.size();
  const int npts = rp_npts(c->k);
  std::vector<RpPass> P(m);
  std::vector<int32_t*> d_status(m, nullptr);
  std::vector<size_t> Bs(m, 0);
  rc.assign(m, FTS_API_OK);
  // per group: its requests with range proofs (the caller batches of the pass, in
  // pass order), their first proof, and the sigma-exclusion hook of its action calls
  std::vector<std::vector<RpReq*>> rpq(m);
  std::vector<std::vector<int>> first(m);
  std::vector<SigHook> hooks(m);
  std::vector<uint8_t> sig_only(m, 0);
  for (size_t j = 0; j < m; j++) {
    Lane& L = *lanes[j];
    const std::vector<RpReq*>& grp = sub[j];
    for (RpReq* q : grp)
      if (q->b->B > 0) rpq[j].push_back(q);
    auto enq = [&]() -> int {
      if (grp.size() == 1 && !grp[0]->act) {
        fts_rp_batch* b = grp[0]->b;
        HIP_OK(hipMemcpyAsync(b->status, b->status0, (size_t)b->B * 4, hipMemcpyDeviceToDevice, L.s));
        Bs[j] = (size_t)b->B;
        d_status[j] = b->status;
        first[j] = {0};
        return rp_enqueue(c, L, b->B, b->raw, b->sc, b->status, b->ipa_flag, [] {}, std::vector<int>{0, b->B}, P[j],
                          nullptr, nullptr);
      }
      size_t B = 0;
      for (RpReq* q : rpq[j]) B += (size_t)q->b->B;
      Workspace& w = L.ws;
      L.tl.begin(L.s);  // the gather on the pass's timeline
      P[j].tl_started = true;
      // the action calls' sigma decode (their slots' streams, since staging) wrote the
      // V slots of their range proofs: the gather waits for that part only; the sigma
      // equations are waited for by the exclusion hook, on the batch check's stream
      for (RpReq* q : grp)
        if (q->act) HIP_OK(hipStreamWaitEvent(L.s, q->act->ev_sig[1], 0));
      RpGather g{};
      if (B > 0) {
        const size_t Bal = std::max(B, std::min(c->coalesce_max, (size_t)1 << 20));  // sized once for the largest pass
        if (w.rp_raw.ensure(Bal * npts * 64) || w.rp_sc.ensure(Bal * RP_NSC * 32) || w.rp_status.ensure(Bal * 4) ||
            w.rp_ipa.ensure(Bal * 4))
          return FTS_API_ENOMEM;
        g.G = (int)rpq[j].size();
        size_t off = 0;
        for (int i = 0; i < g.G; i++) {
          const fts_rp_batch* b = rpq[j][i]->b;
          g.raw[i] = b->raw;
          g.sc[i] = b->sc;
          g.status0[i] = b->status0;
          g.ipa[i] = b->ipa_flag;
          g.off[i] = (int)off;
          first[j].push_back((int)off);
          off += (size_t)b->B;
        }
        g.off[g.G] = (int)off;
        launch_rp_gather(g, c->k, w.rp_raw.as<uint8_t>(), w.rp_sc.as<uint32_t>(), w.rp_status.as<int32_t>(),
                         w.rp_ipa.as<int32_t>(), L.s);
        L.tl.mark("k_rp_gather", L.s, 0);
      }
      Bs[j] = B;
      d_status[j] = w.rp_status.as<int32_t>();
      // the batch check's variable part drops the range proofs of actions whose sigma
      // proof failed (k_sig_exclude at the call's pass offset, on the check's stream, which
      // follows the main stream and so the sigma events)
      SigHook& h = hooks[j];
      h.L = &L;
      for (RpReq* q : grp) {
        if (!q->act || q->act->sd.A == 0) continue;
        int off = -1;
        for (size_t i = 0; i < rpq[j].size(); i++)
          if (rpq[j][i] == q) off = first[j][i];
        h.sig.push_back(&q->act->sd);
        h.off.push_back(off);
        h.ev.push_back(q->act->ev_sig[2]);
      }
      if (B == 0) {  // sigma proofs only: nothing left for the pass but the verdicts
        sig_only[j] = 1;
        for (hipEvent_t e : h.ev) HIP_OK(hipStreamWaitEvent(L.s, e, 0));
        return FTS_API_OK;
      }
      void (*pre)(void*, hipStream_t) = nullptr;
      if (!h.sig.empty()) {
        pre = [](void* arg, hipStream_t s) {
          SigHook* hk = static_cast<SigHook*>(arg);
          // the mask is read at launch time: rp_enqueue sizes (and may re-allocate) it
          for (size_t i = 0; i < hk->sig.size(); i++) {
            (void)hipStreamWaitEvent(s, hk->ev[i], 0);  // the call's sigma verdicts
            if (hk->off[i] >= 0) launch_sig_exclude(*hk->sig[i], hk->L->ws.rp_excl.as<int32_t>() + hk->off[i], s);
          }
        };
      }
      std::vector<int> groups = first[j];
      groups.push_back((int)B);
      return rp_enqueue(c, L, (int)B, w.rp_raw.as<uint8_t>(), w.rp_sc.as<uint32_t>(), w.rp_status.as<int32_t>(),
                        w.rp_ipa.as<int32_t>(), [] {}, groups, P[j], pre, pre ? &h : nullptr);
    };
    rc[j] = enq();
    // the verdicts' downloads behind the pass, before its flag is read: a clean pass
    // (no fallback) needs no second round trip (fin re-downloads after a fallback)
    if (rc[j] == FTS_API_OK && !sig_only[j]) {
      int32_t* pst = L.status_buf(std::max<size_t>(Bs[j], 1));
      if (!pst) {
        rc[j] = FTS_API_ENOMEM;
      } else {
        if (Bs[j] && hipMemcpyAsync(pst, d_status[j], Bs[j] * 4, hipMemcpyDeviceToHost, L.s) != hipSuccess)
          rc[j] = FTS_API_EDEVICE;
        for (RpReq* q : grp)
          if (q->act && q->act->sd.A &&
              hipMemcpyAsync(q->act->sig_res, q->act->sd.status, (size_t)q->act->sd.A * 4, hipMemcpyDeviceToHost,
                             L.s) != hipSuccess)
            rc[j] = FTS_API_EDEVICE;
      }
    }
    for (RpReq* q : rpq[j]) {
      P[j].dense.push_back(q->b->dense ? 1 : 0);
      P[j].bats.push_back(q->b);
    }
  }
  for (size_t j = 0; j < m; j++) {
    Lane& L = *lanes[j];
    if (rc[j] != FTS_API_OK) {
      (void)L.sync();  // drain whatever was enqueued before the failure
      continue;
    }
    auto fin = [&]() -> int {
      if (!sig_only[j]) {
        if (int r = rp_finish(c, L, P[j])) return r;
        for (size_t q = 0; q < rpq[j].size() && q < P[j].dense.size(); q++) rpq[j][q]->b->dense = P[j].dense[q] != 0;
      }
      int32_t* pst = L.status_buf(std::max<size_t>(Bs[j], 1));
      if (!pst) return FTS_API_ENOMEM;
      if (!P[j].clean) {  // a fallback (or a sigma-only pass) ran after the early downloads
        if (Bs[j]) HIP_OK(hipMemcpyAsync(pst, d_status[j], Bs[j] * 4, hipMemcpyDeviceToHost, L.s));
        for (RpReq* q : sub[j])
          if (q->act && q->act->sd.A)
            HIP_OK(hipMemcpyAsync(q->act->sig_res, q->act->sd.status, (size_t)q->act->sd.A * 4, hipMemcpyDeviceToHost,
                                  L.s));
        HIP_OK(L.sync());
      }
      for (size_t i = 0; i < rpq[j].size(); i++) {
        RpReq* q = rpq[j][i];
        const int32_t* v = pst + first[j][i];
        if (q->status) memcpy(q->status, v, (size_t)q->b->B * 4);
        if (P[j].located == 0 && std::any_of(v, v + q->b->B, [](int32_t x) { return x != 0; })) {
          q->b->locate_skip = q->b->locate_backoff;  // a batch of a multi-fault pass that holds bad proofs
          q->b->locate_backoff = std::min(2 * q->b->locate_backoff, 256);
        }
      }
      // host-side timings of the pass: the first action call's parse and staging
      for (RpReq* q : sub[j])
        if (q->act) {
          L.host_parse_ms = q->act->parse_ms;
          L.host_stage_ms = q->act->stage_ms;
          break;
        }
      // the sigma kernels of the pass's first action call (its slot's stream), beside
      const ActSlot* sa = nullptr;
      for (RpReq* q : sub[j])
        if (q->act && q->act->sd.A) {
          sa = q->act;
          break;
        }
      float sig_ms[2] = {0, 0};
      if (sa) {
        (void)hipEventElapsedTime(&sig_ms[0], sa->ev_sig[0], sa->ev_sig[1]);
        (void)hipEventElapsedTime(&sig_ms[1], sa->ev_sig[1], sa->ev_sig[2]);
      }
      for (RpReq* q : sub[j]) {
        collect_timings(c, L, q->b, sa ? sig_ms : nullptr);
        q->b->merged = (int)sub[j].size();
      }
      return FTS_API_OK;
    };
    rc[j] = fin();
  }
}

static int rp_dispatch(fts_ctx* c, RpReq& me);

extern "C" {

// debug/parity hook: intermediates of proof i of the last range-proof run
//   ch_out: (8 + 2k) x 32 bytes canonical BE Fr  [x, x^2, y, y^-1, z, z^2, polEval, x0, x_j.., x_j^-1..]
//   com_out: 64 bytes com (BE) ; hp_out: n x 64 bytes H'_i (BE)
int fts_debug_rp_intermediates(fts_ctx* c, size_t i, uint8_t* ch_out, uint8_t* com_out, uint8_t* hp_out) {
  if (c && !c->shards.empty()) return fts_debug_rp_intermediates(c->shards[0], i, ch_out, com_out, hp_out);
  if (!c || c->device < 0) return FTS_API_EINVAL;
  int want;
  {
    std::lock_guard<std::mutex> g(c->tim_mu);
    want = c->last_lane;
  }
  LaneGuard lg(c, want);
  Workspace& ws = lg.L->ws;
  HIP_OK(hipSetDevice(c->device));
  const int n = c->n, k = c->k, nch = rp_nch(k);
  if (ch_out) {
    std::vector<uint32_t> ch(nch * 8);
    HIP_OK(hipMemcpy(ch.data(), ws.ch.as<uint32_t>() + i * nch * 8, nch * 32, hipMemcpyDeviceToHost));
    for (int q = 0; q < nch; q++) {
      Fr m;
      memcpy(m.v, &ch[q * 8], 32);
      fr_to_be(m, ch_out + 32 * q);
    }
  }
  if (com_out) HIP_OK(hipMemcpy(com_out, ws.hpbe.as<uint8_t>() + (i * (n + 1) + n) * 64, 64, hipMemcpyDeviceToHost));
  if (hp_out) HIP_OK(hipMemcpy(hp_out, ws.hpbe.as<uint8_t>() + i * (n + 1) * 64, n * 64, hipMemcpyDeviceToHost));
  return FTS_API_OK;
}

// debug: bucket-occupancy statistics of the last RLC MSM
// out[0] = max bucket count, out[1] = its bucket index, out[2] = NB, out[3] = #nonzero buckets
int fts_debug_msm_stats(fts_ctx* c, int64_t* out) {
  if (c && !c->shards.empty()) return fts_debug_msm_stats(c->shards[0], out);
  if (!c || c->device < 0 || !out) return FTS_API_EINVAL;
  int want;
  {
    std::lock_guard<std::mutex> g(c->tim_mu);
    want = c->last_lane;
  }
  LaneGuard lg(c, want);
  Workspace& ws = lg.L->ws;
  size_t nb = ws.m_counts.cap / 4;
  std::vector<uint32_t> cnt(nb);
  HIP_OK(hipMemcpy(cnt.data(), ws.m_counts.p, nb * 4, hipMemcpyDeviceToHost));
  size_t arg = 0, nz = 0;
  for (size_t i = 0; i < nb; i++) {
    if (cnt[i] > cnt[arg]) arg = i;
    nz += cnt[i] != 0;
  }
  out[0] = cnt[arg];
  out[1] = (int64_t)arg;
  out[2] = (int64_t)nb;
  out[3] = (int64_t)nz;
  return FTS_API_OK;
}

int fts_rp_batch_stage(fts_ctx* c, size_t n, const uint8_t* const* rp_der, const size_t* rp_len, const uint8_t* com64,
                       fts_rp_batch** out) {
  if (!c || !out || (n && (!rp_der || !rp_len || !com64))) return FTS_API_EINVAL;
  if (!c->shards.empty()) {  // one child batch per device, contiguous shards
    fts_rp_batch* b = new fts_rp_batch();
    b->B = (int)n;
    b->device = c->device;
    b->bounds = plan(n, nullptr, (int)c->shards.size());
    b->parts.assign(c->shards.size(), nullptr);
    b->part_ctx = c->shards;
    int rc = run_shards(b->bounds, [&](int j, size_t lo, size_t hi) {
      return fts_rp_batch_stage(c->shards[j], hi - lo, rp_der + lo, rp_len + lo, com64 + 64 * lo, &b->parts[j]);
    });
    if (rc != FTS_API_OK) {
      fts_rp_batch_free(b);
      return rc;
    }
    *out = b;
    return FTS_API_OK;
  }
  if (c->device < 0) return FTS_API_EDEVICE;
  HIP_OK(hipSetDevice(c->device));
  RpHost h;
  parse_rp_batch(c->k, n, rp_der, rp_len, com64, h);
  fts_rp_batch* b = new fts_rp_batch();
  b->B = (int)n;
  b->device = c->device;
  size_t nb = std::max<size_t>(n, 1);
  if (hipMalloc(&b->raw, std::max<size_t>(h.raw.size(), 64)) != hipSuccess ||
      hipMalloc(&b->sc, std::max<size_t>(h.sc.size() * 4, 32)) != hipSuccess ||
      hipMalloc(&b->status0, nb * 4) != hipSuccess || hipMalloc(&b->status, nb * 4) != hipSuccess ||
      hipMalloc(&b->ipa_flag, nb * 4) != hipSuccess) {
    fts_rp_batch_free(b);
    return FTS_API_ENOMEM;
  }
  if (n) {
    HIP_OK(hipMemcpy(b->raw, h.raw.data(), h.raw.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(b->sc, h.sc.data(), h.sc.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(b->status0, h.status.data(), n * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(b->ipa_flag, h.ipa.data(), n * 4, hipMemcpyHostToDevice));
  }
  *out = b;
  return FTS_API_OK;
}

int fts_rp_batch_verify(fts_ctx* c, fts_rp_batch* b, int32_t* status) {
  if (!c || !b) return FTS_API_EINVAL;
  if (!b->parts.empty()) {
    if (c->shards != b->part_ctx) return FTS_API_EINVAL;  // staged on another context
    int m = 0;
    int rc = run_shards(b->bounds, [&](int j, size_t lo, size_t hi) {
      return fts_rp_batch_verify(c->shards[j], b->parts[j], status ? status + lo : nullptr);
    });
    for (fts_rp_batch* q : b->parts)
      if (q) m = std::max(m, q->merged);
    b->merged = m;
    return rc;
  }
  if (c->device < 0) return FTS_API_EDEVICE;
  if (b->B == 0) return FTS_API_OK;
  HIP_OK(hipSetDevice(c->device));
  RpReq me(b, status);
  return rp_dispatch(c, me);
}

}  // extern "C"

// Work-sharing dispatcher: the request joins the pending queue; any waiting
// caller that finds a free lane takes the queue's head group (FIFO, up to
// coalesce_max proofs) and runs it as ONE device pass, so batches submitted
// while the lanes are busy are merged (a 4,096-proof batch alone fills only
// 64 waves in the per-proof chain kernels).  Verdicts stay per proof.  Staged
// range-proof batches and action calls share the queue and the passes.
static int rp_dispatch(fts_ctx* c, RpReq& me) {
  fts_rp_batch* b = me.b;
  std::unique_lock<std::mutex> lk(c->mu);
  c->rp_pending.push_back(&me);
  c->pending_proofs += (size_t)b->B;
  // a lone arrival: nothing else arrived within the quiet gap before it
  const bool lone = me.arrived - c->last_arrival > std::chrono::microseconds(c->idle_quiet_us);
  c->last_arrival = me.arrived;
  c->arrivals++;
  // enough queued for a full pass: the head stops gathering
  if (c->pending_proofs >= c->gather_target && c->rp_pending.front() != &me) c->rp_pending.front()->cv.notify_one();
  if (c->hold_n > 0 && (int)c->rp_pending.size() >= c->hold_n) {  // test hook: release the held queue
    c->hold_n = 0;
    for (RpReq* q : c->rp_pending) q->cv.notify_one();
  }
  while (!me.done) {
    if (c->free_lanes.empty() || c->rp_pending.empty() || c->hold_n > 0) {
      me.cv.wait(lk);
      continue;
    }
    const bool device_busy = c->free_lanes.size() < c->lanes.size();
    const int wait_us = device_busy ? c->gather_us : c->idle_gather_us;
    if (wait_us > 0 && c->rp_pending.front() == &me && c->pending_proofs < c->gather_target) {
      auto deadline = me.arrived + std::chrono::microseconds(wait_us);
      if (!device_busy) {  // idle: only while the burst is still arriving
        deadline = std::min(deadline, c->last_arrival + std::chrono::microseconds(c->idle_quiet_us));
        if (lone && c->rp_pending.size() == 1) {
          // a lone caller: a short spin for company, then go (no wake-up latency)
          deadline = std::min(deadline, me.arrived + std::chrono::microseconds(c->idle_first_us));
          if (std::chrono::steady_clock::now() < deadline) {
            const uint64_t a0 = c->arrivals.load();
            lk.unlock();
            while (std::chrono::steady_clock::now() < deadline && c->arrivals.load() == a0) std::this_thread::yield();
            lk.lock();
            continue;
          }
        }
      }
      if (std::chrono::steady_clock::now() < deadline) {
        me.cv.wait_until(lk, deadline);
        continue;
      }
    }
    if (c->rp_pending.front() != &me && !me.done) {  // only the head leads a pass
      c->rp_pending.front()->cv.notify_one();
      me.cv.wait(lk);
      continue;
    }
    Lane* L = c->lanes[c->free_lanes.back()];
    c->free_lanes.pop_back();
    L->alone = c->free_lanes.size() + 1 == c->lanes.size();
    // an idle device's first pass stops at gather_target proofs (the rest of the
    // burst forms the next pass on another lane)
    const size_t cap = L->alone ? std::min(c->coalesce_max, std::max<size_t>(c->gather_target, 1)) : c->coalesce_max;
    std::vector<RpReq*> grp;
    size_t tot = 0;
    while (!c->rp_pending.empty()) {
      RpReq* q = c->rp_pending.front();
      if (!grp.empty() && (tot + (size_t)q->b->B > cap || (int)grp.size() == RP_GATHER_MAX)) break;
      grp.push_back(q);
      tot += (size_t)q->b->B;
      c->pending_proofs -= (size_t)q->b->B;
      c->rp_pending.pop_front();
    }
    std::vector<Lane*> lanes{L};
    std::vector<std::vector<RpReq*>> sub{grp};
    // the next head (if any) may lead a pass on another free lane
    if (!c->rp_pending.empty() && !c->free_lanes.empty()) c->rp_pending.front()->cv.notify_one();
    lk.unlock();
    std::vector<int> rcs;
    run_rp_groups(c, lanes, sub, rcs);
    c->st_passes++;
    c->st_reqs += (int64_t)grp.size();
    c->st_act_reqs += std::count_if(grp.begin(), grp.end(), [](const RpReq* q) { return q->act != nullptr; });
    for (int64_t mx = c->st_max_merged.load(); (int64_t)grp.size() > mx && !c->st_max_merged.compare_exchange_weak(mx, (int64_t)grp.size());) {
    }
    lk.lock();
    for (size_t j = 0; j < sub.size(); j++)
      for (RpReq* q : sub[j]) {
        q->rc = rcs[j];
        q->done = true;
        if (q != &me) q->cv.notify_one();
      }
    for (Lane* x : lanes) c->free_lanes.push_back(x->id);
    c->wake_lane_waiters();
  }
  return me.rc;
}

extern "C" {

int fts_rp_batch_timings(const fts_rp_batch* b, const char** names, float* ms, double* mads, int cap) {
  if (!b) return 0;
  if (!b->parts.empty()) return b->parts[0] ? fts_rp_batch_timings(b->parts[0], names, ms, mads, cap) : 0;
  int m = std::min(cap, b->ntim);
  for (int i = 0; i < m; i++) {
    if (names) names[i] = b->tim_name[i];
    if (ms) ms[i] = b->tim_ms[i];
    if (mads) mads[i] = b->tim_work[i] * MADS_PER_MUL;
  }
  return m;
}

int fts_rp_batch_merged(const fts_rp_batch* b) { return b ? b->merged : 0; }

int fts_debug_hold(fts_ctx* c, int n) {
  if (!c) return FTS_API_EINVAL;
  for (fts_ctx* ch : c->shards) fts_debug_hold(ch, n);
  if (c->lanes.empty()) return FTS_API_OK;
  std::lock_guard<std::mutex> g(c->mu);
  c->hold_n = std::max(0, n);
  if (c->hold_n == 0 || (int)c->rp_pending.size() >= c->hold_n) {
    c->hold_n = 0;
    for (RpReq* q : c->rp_pending) q->cv.notify_one();
  }
  return FTS_API_OK;
}

int fts_debug_dispatch_stats(const fts_ctx* c, int64_t* out) {
  if (!c || !out) return FTS_API_EINVAL;
  if (!c->shards.empty()) return fts_debug_dispatch_stats(c->shards[0], out);
  out[0] = c->st_passes.load();
  out[1] = c->st_reqs.load();
  out[2] = c->st_max_merged.load();
  out[3] = c->st_act_reqs.load();
  return FTS_API_OK;
}

int fts_ctx_reserve(fts_ctx* c, size_t max_pass_proofs) {
  if (!c) return FTS_API_EINVAL;
  if (!c->shards.empty()) {
    std::vector<size_t> all(c->shards.size() + 1);
    for (size_t j = 0; j < all.size(); j++) all[j] = j;  // one "item" per device
    return run_shards(all, [&](int j, size_t, size_t) { return fts_ctx_reserve(c->shards[j], max_pass_proofs); });
  }
  if (c->device < 0) return FTS_API_EDEVICE;
  const size_t B = max_pass_proofs ? max_pass_proofs : c->coalesce_max;
  if (B == 0 || B > (1u << 20)) return FTS_API_ESIZE;
  HIP_OK(hipSetDevice(c->device));
  for (size_t i = 0; i < c->lanes.size(); i++) {
    LaneGuard lg(c, (int)i);
    if (int rc = lane_reserve(c, *lg.L, (int)B, true)) return rc;
    HIP_OK(lg.L->sync());
  }
  return FTS_API_OK;
}

// ------------------------------------------------- standalone G1 MSM (C3)
}  // extern "C"
struct fts_msm_batch {
  int N = 0;
  int device = 0;
  uint32_t* pts = nullptr;  // [N][16] affine Montgomery
  uint32_t* sc = nullptr;   // [N][8] canonical scalars
  uint8_t* out = nullptr;   // 64-byte result
  int ntim = 0;
  const char* tim_name[Timeline::CAP];
  float tim_ms[Timeline::CAP];
  double tim_work[Timeline::CAP];
};
extern "C" {

void fts_msm_free(fts_msm_batch* b) {
  if (!b) return;
  hipSetDevice(b->device);
  for (void* p : {(void*)b->pts, (void*)b->sc, (void*)b->out})
    if (p) hipFree(p);
  delete b;
}

int fts_msm_stage(fts_ctx* c, size_t n, const uint8_t* points64, const uint8_t* scalars32, fts_msm_batch** out) {
  if (c && !c->shards.empty()) return fts_msm_stage(c->shards[0], n, points64, scalars32, out);
  if (!c || !out || !n || !points64 || !scalars32 || n > (size_t)(1u << 26)) return FTS_API_EINVAL;
  if (c->device < 0) return FTS_API_EDEVICE;
  HIP_OK(hipSetDevice(c->device));
  fts_msm_batch* b = new fts_msm_batch();
  b->N = (int)n;
  b->device = c->device;
  uint8_t *rp = nullptr, *rs = nullptr;
  uint32_t* bad = nullptr;
  if (hipMalloc(&b->pts, n * 64) != hipSuccess || hipMalloc(&b->sc, n * 32) != hipSuccess ||
      hipMalloc(&b->out, 64) != hipSuccess || hipMalloc(&rp, n * 64) != hipSuccess || hipMalloc(&rs, n * 32) != hipSuccess ||
      hipMalloc(&bad, 4) != hipSuccess) {
    for (void* p : {(void*)rp, (void*)rs, (void*)bad})
      if (p) hipFree(p);
    fts_msm_free(b);
    return FTS_API_ENOMEM;
  }
  uint32_t nbad = 0;
  hipError_t e = hipMemcpy(rp, points64, n * 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(rs, scalars32, n * 32, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(bad, 0, 4);
  if (e == hipSuccess) {
    launch_msm_load((int)n, rp, rs, b->pts, b->sc, bad, 0);
    e = hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost);
  }
  hipFree(rp);
  hipFree(rs);
  hipFree(bad);
  if (e != hipSuccess) {
    fts_msm_free(b);
    return FTS_API_EDEVICE;
  }
  if (nbad) {  // a point failed NewG1FromBytes (flags, range, on-curve)
    fts_msm_free(b);
    return FTS_API_EINVAL;
  }
  *out = b;
  return FTS_API_OK;
}

int fts_msm_stage_multiples(fts_ctx* c, size_t n, const uint8_t* k32, const uint8_t* scalars32, fts_msm_batch** out) {
  if (c && !c->shards.empty()) return fts_msm_stage_multiples(c->shards[0], n, k32, scalars32, out);
  if (!c || !out || !n || !k32 || !scalars32 || n > (size_t)(1u << 26)) return FTS_API_EINVAL;
  if (c->device < 0) return FTS_API_EDEVICE;
  HIP_OK(hipSetDevice(c->device));
  fts_msm_batch* b = new fts_msm_batch();
  b->N = (int)n;
  b->device = c->device;
  if (hipMalloc(&b->pts, n * 64) != hipSuccess || hipMalloc(&b->sc, n * 32) != hipSuccess ||
      hipMalloc(&b->out, 64) != hipSuccess) {
    fts_msm_free(b);
    return FTS_API_ENOMEM;
  }
  // the temporaries on a private stream with stream-ordered allocation, synchronised
  // alone: a device-wide sync (hipDeviceSynchronize, or hipFree) here would stall
  // every lane's in-flight pass on a shared context
  uint8_t *rk = nullptr, *rs = nullptr;
  uint32_t* jac = nullptr;
  hipStream_t st = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMallocAsync((void**)&rk, n * 32, st);
  if (e == hipSuccess) e = hipMallocAsync((void**)&rs, n * 32, st);
  if (e == hipSuccess) e = hipMallocAsync((void**)&jac, n * 96, st);
  if (e == hipSuccess) e = hipMemcpyAsync(rk, k32, n * 32, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(rs, scalars32, n * 32, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    // B = the PP's ped[1] (table slot tb_G): a generator of G1
    launch_msm_gen_points((int)n, rk, rs, c->d_tables + (size_t)tb_G(c->n) * fb_words_per_base(), jac, b->pts, b->sc,
                          st);
    e = hipGetLastError();
  }
  for (void* p : {(void*)rk, (void*)rs, (void*)jac})
    if (p) (void)hipFreeAsync(p, st);
  if (st) {
    const hipError_t e2 = hipStreamSynchronize(st);
    if (e == hipSuccess) e = e2;
    hipStreamDestroy(st);
  }
  if (e != hipSuccess) {
    fts_msm_free(b);
    return e == hipErrorOutOfMemory ? FTS_API_ENOMEM : FTS_API_EDEVICE;
  }
  *out = b;
  return FTS_API_OK;
}

int fts_msm_points(fts_ctx* c, const fts_msm_batch* b, size_t lo, size_t count, uint8_t* out64) {
  if (c && !c->shards.empty()) return fts_msm_points(c->shards[0], b, lo, count, out64);
  if (!c || !b || (count && !out64) || lo > (size_t)b->N || count > (size_t)b->N - lo) return FTS_API_EINVAL;
  if (c->device < 0) return FTS_API_EDEVICE;
  if (!count) return FTS_API_OK;
  HIP_OK(hipSetDevice(c->device));
  // private stream and stream-ordered scratch: no device-wide sync (see fts_msm_stage_multiples)
  hipStream_t st = nullptr;
  uint8_t* d = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMallocAsync((void**)&d, count * 64, st);
  if (e == hipSuccess) {
    launch_msm_pts_to_bytes((int)count, b->pts + lo * 16, d, st);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out64, d, count * 64, hipMemcpyDeviceToHost, st);
  if (d) (void)hipFreeAsync(d, st);
  if (st) {
    const hipError_t e2 = hipStreamSynchronize(st);
    if (e == hipSuccess) e = e2;
    hipStreamDestroy(st);
  }
  return e == hipSuccess ? FTS_API_OK : FTS_API_EDEVICE;
}

int fts_msm_run(fts_ctx* c, fts_msm_batch* b, uint8_t* out64) {
  if (c && !c->shards.empty()) return fts_msm_run(c->shards[0], b, out64);
  if (!c || !b || !out64) return FTS_API_EINVAL;
  if (c->device < 0) return FTS_API_EDEVICE;
  HIP_OK(hipSetDevice(c->device));
  LaneGuard lg(c);
  Lane& L = *lg.L;
  MsmPlan mp{};
  // standalone MSMs: the block-local counting sort; from 2^20 points 32-point
  // chunks (~8 partials per bucket instead of ~32 at 2^22)
  if (int rc = msm_prepare(L, b->N, mp, MSM_SLOT_PASS, b->N >= (1 << 20) ? 32 : MSM_CH, c->msm_sort != 0, c->msm_maxc))
    return rc;
  L.tl.begin(L.s);
  launch_msm(mp, b->pts, b->sc, nullptr, 0, L.ws.m_scratch.as<uint32_t>(), L.s, L.s, &L.tl);
  launch_msm_to_bytes(mp.out, b->out, L.s);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(out64, b->out, 64, hipMemcpyDeviceToHost, L.s));
  HIP_OK(L.sync());
  b->ntim = 0;
  for (int i = 0; i < L.tl.n && b->ntim < Timeline::CAP; i++) {
    if (!L.tl.name[i]) continue;
    const int j = b->ntim++;
    b->tim_name[j] = L.tl.name[i];
    b->tim_work[j] = L.tl.work[i];
    hipEventElapsedTime(&b->tim_ms[j], L.tl.ev[L.tl.start[i]], L.tl.ev[i + 1]);
  }
  return FTS_API_OK;
}

int fts_msm_timings(const fts_msm_batch* b, const char** names, float* ms, double* mads, int cap) {
  if (!b) return 0;
  int m = std::min(cap, b->ntim);
  for (int i = 0; i < m; i++) {
    if (names) names[i] = b->tim_name[i];
    if (ms) ms[i] = b->tim_ms[i];
    if (mads) mads[i] = b->tim_work[i] * MADS_PER_MUL;
  }
  return m;
}

int fts_msm_g1(fts_ctx* c, size_t n, const uint8_t* points64, const uint8_t* scalars32, uint8_t* out64) {
  if (!out64) return FTS_API_EINVAL;
  if (n == 0) {
    memset(out64, 0, 64);
    return FTS_API_OK;
  }
  if (c && !c->shards.empty()) {
    // partial MSM per device, the partial points combined on the host
    const std::vector<size_t> bnd = plan(n, nullptr, (int)c->shards.size());
    std::vector<uint8_t> part(64 * c->shards.size(), 0);
    int rc = run_shards(bnd, [&](int j, size_t lo, size_t hi) {
      return fts_msm_g1(c->shards[j], hi - lo, points64 + 64 * lo, scalars32 + 32 * lo, &part[64 * j]);
    });
    if (rc != FTS_API_OK) return rc;
    G1J acc = jac_identity();
    for (size_t j = 0; j < c->shards.size(); j++) {
      G1A a;
      if (!g1_from_bytes(&part[64 * j], 64, a)) return FTS_API_EDEVICE;
      acc = jadd_aff(acc, a);
    }
    g1_to_bytes(to_aff(acc), out64);
    return FTS_API_OK;
  }
  fts_msm_batch* b = nullptr;
  int rc = fts_msm_stage(c, n, points64, scalars32, &b);
  if (rc != FTS_API_OK) return rc;
  rc = fts_msm_run(c, b, out64);
  fts_msm_free(b);
  return rc;
}

void fts_rp_batch_free(fts_rp_batch* b) {
  if (!b) return;
  if (!b->parts.empty() || !b->part_ctx.empty()) {
    for (fts_rp_batch* q : b->parts) fts_rp_batch_free(q);
    delete b;
    return;
  }
  hipSetDevice(b->device);
  for (void* p : {(void*)b->raw, (void*)b->sc, (void*)b->status0, (void*)b->status, (void*)b->ipa_flag})
    if (p) hipFree(p);
  delete b;
}

// a staging slot sized for n proofs (idle one reused, else a new one); nullptr on
// allocation failure
static RpSlot* slot_acquire(fts_ctx* c, size_t n) {
  RpSlot* sl = nullptr;
  {
    std::lock_guard<std::mutex> g(c->slot_mu);
    if (!c->free_slots.empty()) {
      sl = c->free_slots.back();
      c->free_slots.pop_back();
    }
  }
  if (!sl) {
    sl = new RpSlot();
    sl->b = new fts_rp_batch();
    sl->b->device = c->device;
    if (hipStreamCreateWithFlags(&sl->s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&sl->done, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess) {
      if (sl->s) hipStreamDestroy(sl->s);
      delete sl->b;
      delete sl;
      return nullptr;
    }
    std::lock_guard<std::mutex> g(c->slot_mu);
    c->slots.push_back(sl);
  }
  const size_t npts = (size_t)rp_npts(c->k);
  const size_t in_bytes = n * (npts * 64 + RP_NSC * 32 + 8), dev_bytes = in_bytes + n * 4;
  bool ok = true;
  if (in_bytes > sl->pin_cap) {
    if (sl->pin) (void)hipHostFree(sl->pin);
    sl->pin = nullptr;
    const size_t want = std::max(in_bytes, sl->pin_cap + sl->pin_cap / 2);
    sl->pin_cap = 0;
    if (hipHostMalloc((void**)&sl->pin, want, 0) == hipSuccess) sl->pin_cap = want;
    else ok = false;
  }
  if (ok && dev_bytes > sl->dev_cap) {
    if (sl->dev) hipFree(sl->dev);
    sl->dev = nullptr;
    const size_t want = std::max(dev_bytes, sl->dev_cap + sl->dev_cap / 2);
    sl->dev_cap = 0;
    if (hipMalloc((void**)&sl->dev, want) == hipSuccess) sl->dev_cap = want;
    else ok = false;
  }
  if (!ok) {
    std::lock_guard<std::mutex> g(c->slot_mu);
    c->free_slots.push_back(sl);
    return nullptr;
  }
  return sl;
}

int fts_rp_verify_batch(fts_ctx* c, size_t n, const uint8_t* const* rp_der, const size_t* rp_len, const uint8_t* com64,
                        int32_t* status) {
  if (!c || !status) return FTS_API_EINVAL;
  if (n == 0) return FTS_API_OK;
  if (!rp_der || !rp_len || !com64) return FTS_API_EINVAL;
  if (!c->shards.empty()) return multi_rp_verify(c, n, rp_der, rp_len, com64, status);
  auto not_run = [&](int rc) {
    for (size_t i = 0; i < n; i++) status[i] = FTS_E_NOT_RUN;
    return rc;
  };
  if (c->device < 0) return not_run(FTS_API_EDEVICE);
  if (n > (size_t)INT32_MAX) return not_run(FTS_API_ESIZE);
  if (hipSetDevice(c->device) != hipSuccess) return not_run(FTS_API_EDEVICE);
  // host DER -> pinned records (parallel), one async upload on the slot's stream,
  // then the staged batch joins the coalescing dispatcher like any other
  RpSlot* sl = slot_acquire(c, n);
  if (!sl) return not_run(FTS_API_ENOMEM);
  const size_t npts = (size_t)rp_npts(c->k);
  const size_t raw_b = n * npts * 64, sc_b = n * RP_NSC * 32, st_b = n * 4;
  uint8_t* p = sl->pin;
  parse_rp_into(c->k, n, rp_der, rp_len, com64, p, reinterpret_cast<uint32_t*>(p + raw_b),
                reinterpret_cast<int32_t*>(p + raw_b + sc_b), reinterpret_cast<int32_t*>(p + raw_b + sc_b + st_b));
  fts_rp_batch* b = sl->b;
  // the slot's batch object serves unrelated callers in turn: the adaptive
  // group-test state (FTS_GT_ADAPT) is per caller batch, so an honest call never
  // inherits the dense schedule of the previous caller's tampered one
  b->dense = false;
  b->locate_skip = 0, b->locate_backoff = 8;
  b->merged = 1;
  b->ntim = 0;
  b->B = (int)n;
  b->raw = sl->dev;
  b->sc = reinterpret_cast<uint32_t*>(sl->dev + raw_b);
  b->status0 = reinterpret_cast<int32_t*>(sl->dev + raw_b + sc_b);
  b->ipa_flag = reinterpret_cast<int32_t*>(sl->dev + raw_b + sc_b + st_b);
  b->status = reinterpret_cast<int32_t*>(sl->dev + raw_b + sc_b + 2 * st_b);
  int rc = FTS_API_OK;
  if (hipMemcpyAsync(sl->dev, sl->pin, raw_b + sc_b + 2 * st_b, hipMemcpyHostToDevice, sl->s) != hipSuccess ||
      hipEventRecord(sl->done, sl->s) != hipSuccess || hipEventSynchronize(sl->done) != hipSuccess)
    rc = FTS_API_EDEVICE;
  if (rc == FTS_API_OK) rc = fts_rp_batch_verify(c, b, status);
  else not_run(rc);
  {
    std::lock_guard<std::mutex> g(c->slot_mu);
    c->free_slots.push_back(sl);
  }
  return rc;
}


// ------------------------------------------------------- transfers / issues
// One action = a transfer (TypeAndSum + RangeCorrectness on Out_j - CT,
// transfer/transfer.go:49-60,153-197) or an issue (SameType + RangeCorrectness
// on Tok_i - CT, issue/verifier.go:24-57).  An action call is parsed straight into
// a pooled slot's pinned records (act_stage), uploaded once, and verified by the
// range-proof dispatcher (rp_dispatch) together with whatever else is queued.

// an idle action staging slot (or a new one); nullptr on failure
static ActSlot* aslot_acquire(fts_ctx* c) {
  {
    std::lock_guard<std::mutex> g(c->slot_mu);
    if (!c->free_aslots.empty()) {
      ActSlot* sl = c->free_aslots.back();
      c->free_aslots.pop_back();
      return sl;
    }
  }
  ActSlot* sl = new ActSlot();
  sl->b = new fts_rp_batch();
  sl->b->device = c->device;
  if (hipStreamCreateWithFlags(&sl->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&sl->done, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&sl->ev_sig[0]) != hipSuccess || hipEventCreate(&sl->ev_sig[1]) != hipSuccess ||
      hipEventCreate(&sl->ev_sig[2]) != hipSuccess) {
    for (hipEvent_t e : sl->ev_sig)
      if (e) hipEventDestroy(e);
    if (sl->done) hipEventDestroy(sl->done);
    if (sl->s) hipStreamDestroy(sl->s);
    delete sl->b;
    delete sl;
    return nullptr;
  }
  std::lock_guard<std::mutex> g(c->slot_mu);
  c->aslots.push_back(sl);
  return sl;
}

static void aslot_release(fts_ctx* c, ActSlot* sl) {
  std::lock_guard<std::mutex> g(c->slot_mu);
  c->free_aslots.push_back(sl);
}

// grow the slot's pinned and device buffers geometrically (hipFree synchronises the
// whole device: a slot must not be re-allocated on every slightly larger call)
static bool aslot_size(ActSlot* sl, size_t pin_bytes, size_t dev_bytes) {
  if (pin_bytes > sl->pin_cap) {
    if (sl->pin) (void)hipHostFree(sl->pin);
    sl->pin = nullptr;
    const size_t want = std::max(pin_bytes, sl->pin_cap + sl->pin_cap / 2);
    sl->pin_cap = 0;
    if (hipHostMalloc((void**)&sl->pin, want, 0) != hipSuccess) return false;
    sl->pin_cap = want;
  }
  if (dev_bytes > sl->dev_cap) {
    if (sl->dev) hipFree(sl->dev);
    sl->dev = nullptr;
    const size_t want = std::max(dev_bytes, sl->dev_cap + sl->dev_cap / 2);
    sl->dev_cap = 0;
    if (hipMalloc((void**)&sl->dev, want) != hipSuccess) return false;
    sl->dev_cap = want;
  }
  return true;
}

// Parse an action call into slot sl: sigma batch + range-proof records in their
// device layout, written straight into the slot's pinned buffer (no per-action
// host vectors, no second copy), then one upload.  Three steps:
//   1. (parallel) the proofs' outer structure: which actions reach the device and
//      how many range proofs each carries -- the layout's only inputs;
//   2. (serial) offsets of every action's records (integer prefix sums);
//   3. (parallel) the full decode into those offsets.  An action rejected here keeps
//      its records in the layout, marked so every kernel skips them (sigma status
//      FTS_E_MALFORMED, its range proofs FTS_E_NOT_RUN); its verdict is the host's.
// The per-action checks and their order are the reference's deserialisation
// (transfer.go:29-40, typeandsum.go:37-93,230-251, sametype.go:32-64,167-171,
// rangecorrectness.go:19-40, bulletproof.go:37-101, ipa.go:33-67).
static int act_stage(fts_ctx* c, ActSlot* sl, const std::vector<ActionIn>& acts) {
  const double t0 = now_ms();
  const int k = c->k, npts_rp = rp_npts(k);
  const size_t A = acts.size();
  std::vector<ActionState>& st = sl->st;
  st.assign(A, ActionState{});
  // Steps 1 and 3 run over chunks of CH consecutive actions; step 2 scans the
  // chunks' totals only (a serial pass over every action re-read the per-action
  // state the parse threads had just written: ~0.1 us per action of cache-line
  // transfers), and step 3 lays its chunk out from the chunk's base.
  constexpr size_t CH = 128;
  const size_t nch = (A + CH - 1) / CH;
  struct Run {
    int sa = 0, pt = 0, sc = 0, term = 0, nfix = 0, aff = 0, rp = 0;
    uint32_t msg = 0;
    // advance past action (kind, n_in, n_out) with nrp slotted range proofs
    void add(int kind, int n_in, int n_out, int nrp) {
      sa++;
      pt += 1 + n_in + n_out;
      sc += sig_nscalars(kind, n_in);
      term += sig_nterms(kind, n_in);
      nfix += sig_nfixed(kind, n_in);
      aff += sig_naff(kind, n_in, n_out);
      msg += sig_msg_slot(kind, n_in, n_out);
      rp += nrp;
    }
  };
  std::vector<Run> base(nch);
  // ---- 1. shapes, and each chunk's totals
  parallel_for(nch, 2, [&](size_t q) {
    thread_local std::vector<der::Span> vals, rps;
    Run t;
    for (size_t i = q * CH; i < std::min(A, (q + 1) * CH); i++) {
      const ActionIn& ai = acts[i];
      ActionState& s = st[i];
      if (!der::unmarshal_values(ai.proof, vals) || vals.size() != 2) {
        s.host_final = FTS_E_MALFORMED;
        continue;
      }
      s.rc_applicable = ai.kind == SIG_ST || ai.n_in != 1 || ai.n_out != 1;
      rps.clear();
      if (vals[1].n && !parse_range_correctness(vals[1], rps)) {
        s.host_final = FTS_E_MALFORMED;
        continue;
      }
      s.rp_count = (int)rps.size();
      const int n_in = ai.kind == SIG_TAS ? (int)ai.n_in : 0;
      t.add(ai.kind, n_in, (int)ai.n_out, s.rc_applicable ? s.rp_count : 0);
    }
    base[q] = t;
  });
  const double t_p1 = now_ms();
  // ---- 2. chunk bases (exclusive scan) and the totals
  Run tot;
  for (size_t q = 0; q < nch; q++) {
    const Run t = base[q];
    base[q] = tot;
    tot.sa += t.sa, tot.pt += t.pt, tot.sc += t.sc, tot.term += t.term, tot.nfix += t.nfix, tot.aff += t.aff;
    tot.rp += t.rp, tot.msg += t.msg;
  }
  const int SA = tot.sa, pt_off = tot.pt, sc_off = tot.sc, term_off = tot.term, nfix_total = tot.nfix,
            aff_off = tot.aff, rp_total = tot.rp;
  const uint32_t msg_off = tot.msg;
  const size_t nwork = (size_t)term_off;
  size_t o = 0;
  auto region = [&](size_t bytes) {  // 256-byte aligned regions
    size_t r = o;
    o += (bytes + 255) & ~size_t(255);
    return r;
  };
  // uploaded part (one copy), then the pinned verdict download, then device workspace
  const size_t o_act = region((size_t)SA * sizeof(SigAction)), o_raw = region((size_t)pt_off * 64),
               o_owner = region((size_t)pt_off * 4), o_sc = region((size_t)sc_off * 32),
               o_work = region(nwork * sizeof(int2)), o_affoff = region((size_t)SA * 4), o_sst = region((size_t)SA * 4),
               o_rraw = region((size_t)rp_total * npts_rp * 64), o_rsc = region((size_t)rp_total * RP_NSC * 32),
               o_rst = region((size_t)rp_total * 4), o_ripa = region((size_t)rp_total * 4);
  const size_t in_end = o;
  const size_t o_res = region((size_t)SA * 4), pin_end = o;
  o = in_end;
  const size_t w_pts = region((size_t)pt_off * 64), w_terms = region(nwork * 96), w_aff = region((size_t)aff_off * 64),
               w_jac = region((size_t)aff_off * 96), w_msgs = region(msg_off),
               w_scratch = region(sig_scratch_words(nwork) * 4), dev_end = o;
  uint8_t* hp;
  if (c->device < 0) {  // host-only context (fts_debug_stage_actions): the parse alone, into host memory
    sl->host_buf.resize(std::max<size_t>(pin_end, 256));
    hp = sl->host_buf.data();
  } else {
    if (!aslot_size(sl, std::max<size_t>(pin_end, 256), std::max<size_t>(dev_end, 256))) return FTS_API_ENOMEM;
    hp = sl->pin;
  }
  SigAction* hact = reinterpret_cast<SigAction*>(hp + o_act);
  int32_t* hsst = reinterpret_cast<int32_t*>(hp + o_sst);
  int32_t* hrst = reinterpret_cast<int32_t*>(hp + o_rst);
  int32_t* hripa = reinterpret_cast<int32_t*>(hp + o_ripa);
  int32_t* howner = reinterpret_cast<int32_t*>(hp + o_owner);
  int32_t* haffo = reinterpret_cast<int32_t*>(hp + o_affoff);
  int2* hwork = reinterpret_cast<int2*>(hp + o_work);
  // one action: its records at the running offsets, then its decode
  auto decode_one = [&](size_t i, Run& run) {
    thread_local std::vector<der::Span> vals, rps, ubuf, ibf, iv;
    ActionState& s = st[i];
    if (s.host_final >= 0) return;
    const ActionIn& ai = acts[i];
    const int g = run.sa;
    s.sig = g;
    const int n_in = ai.kind == SIG_TAS ? (int)ai.n_in : 0;
    SigAction& sa = hact[g];
    sa = SigAction{};
    sa.kind = ai.kind;
    sa.n_in = n_in;
    sa.n_out = (int)ai.n_out;
    sa.pt_off = run.pt;
    sa.sc_off = run.sc;
    sa.term_off = run.term;
    sa.msg_off = (int32_t)run.msg;
    s.rp_base = s.rc_applicable && s.rp_count > 0 ? run.rp : -1;
    sa.rp_base = s.rp_base;
    sa.rp_count = s.rp_count;
    hsst[g] = 0;
    haffo[g] = run.aff;
    const int npt = 1 + sa.n_in + sa.n_out;
    for (int q = 0; q < npt; q++) howner[sa.pt_off + q] = g;
    // work list: every fixed-base term first, then every variable-base (GLV) term,
    // so each kind has its own kernel (k_sig_fixed, k_sig_var)
    for (int t = 0, nt = sig_nterms(sa.kind, sa.n_in), fi = run.nfix, vi = nfix_total + run.term - run.nfix; t < nt; t++)
      hwork[sig_term_var(sa.kind, sa.n_in, t) ? vi++ : fi++] = make_int2(g, t);
    run.add(ai.kind, n_in, (int)ai.n_out, s.rc_applicable ? s.rp_count : 0);
    // a rejected action keeps its records, skipped by every kernel
    auto fail = [&](int32_t v) {
      s.host_final = v;
      hsst[g] = FTS_E_MALFORMED;
      for (int j = 0; j < s.rp_count && s.rp_base >= 0; j++) {
        hrst[s.rp_base + j] = FTS_E_NOT_RUN;
        hripa[s.rp_base + j] = 0;
      }
    };
    (void)der::unmarshal_values(ai.proof, vals);  // held in step 1
    rps.clear();
    if (vals[1].n) (void)parse_range_correctness(vals[1], rps);
    // ---- range proofs (deserialised together with the sigma proof)
    thread_local std::vector<uint8_t> tpts;
    thread_local std::vector<uint32_t> tsc;
    for (size_t j = 0; j < rps.size(); j++) {
      uint8_t* pts;
      uint32_t* scp;
      int32_t tst = 0, tipa = 0;
      int32_t *pst = &tst, *pipa = &tipa;
      if (s.rp_base >= 0) {
        const size_t r = (size_t)s.rp_base + j;
        pts = hp + o_rraw + r * npts_rp * 64;
        scp = reinterpret_cast<uint32_t*>(hp + o_rsc) + r * RP_NSC * 8;
        pst = hrst + r;
        pipa = hripa + r;
      } else {  // not verified (1-in/1-out transfer), but must deserialise
        tpts.resize((size_t)npts_rp * 64);
        tsc.resize(RP_NSC * 8);
        pts = tpts.data();
        scp = tsc.data();
      }
      parse_range_proof(rps[j], k, pts, scp, *pst, *pipa);
      filler_point(pts + RP_PT_V * 64);
      if (*pst == FTS_E_MALFORMED) return fail(FTS_E_MALFORMED);
      if (!s.rc_applicable) {  // its points decode on the host (no device slot)
        G1A tmp;
        for (int q = 0; q < npts_rp; q++)
          if (q != RP_PT_V && !g1_from_bytes(pts + q * 64, 64, tmp)) return fail(FTS_E_MALFORMED);
      }
    }
    if (s.rc_applicable) s.rc_count_bad = rps.size() != ai.n_out;
    // ---- sigma proof: points [CT, in..., out...], scalars
    uint8_t* raw = hp + o_raw + (size_t)sa.pt_off * 64;
    memset(raw, 0, 64);
    if (sa.n_in) memcpy(raw + 64, ai.in, (size_t)sa.n_in * 64);
    if (ai.n_out) memcpy(raw + (size_t)(1 + sa.n_in) * 64, ai.out, ai.n_out * 64);
    uint32_t* sc = reinterpret_cast<uint32_t*>(hp + o_sc) + (size_t)sa.sc_off * 8;
    memset(sc, 0, (size_t)sig_nscalars(sa.kind, sa.n_in) * 32);
    bool nil_fields = false, panic = false;
    Elem e[7];
    const int ne = ai.kind == SIG_TAS ? 7 : 4;
    if (vals[0].n) {
      Unmarshaller u(vals[0], ubuf);
      if (!u.ok) return fail(FTS_E_MALFORMED);
      for (int f = 0; f < ne; f++)
        if (!u.next(e[f])) return fail(FTS_E_MALFORMED);
    }
    // element kinds: TAS [CT g1, ibf arr, iv arr, Type, TBF, EqSum, Chal]; ST [Type, BF, Chal, CT g1]
    const int ct_idx = ai.kind == SIG_TAS ? 0 : 3;
    if (e[ct_idx].present) {
      if (e[ct_idx].raw.n != 64) return fail(FTS_E_MALFORMED);
      memcpy(raw, e[ct_idx].raw.p, 64);
    }
    if (ai.kind == SIG_TAS) {
      ibf.clear();
      iv.clear();
      if (e[1].present && !der::unmarshal_values(e[1].raw, ibf, true)) return fail(FTS_E_MALFORMED);
      if (e[2].present && !der::unmarshal_values(e[2].raw, iv, true)) return fail(FTS_E_MALFORMED);
      // typeandsum.go:231: nil TBF/Type/CT/EqSum -> "invalid sum and type proof"
      nil_fields = !e[4].present || !e[3].present || !e[0].present || !e[5].present;
      // :242-251 would panic on a nil challenge or short/nil InputValues / InputBlindingFactors
      if (!nil_fields && (!e[6].present || !e[2].present || !e[1].present || iv.size() < ai.n_in || ibf.size() < ai.n_in))
        panic = true;
      // transfer.go:175: the range goroutine dereferences CommitmentToType
      if (s.rc_applicable && !e[0].present) panic = true;
      if (!nil_fields && !panic) {
        scalar_from_bytes(e[3].raw, sc + TAS_SC_TYPE * 8, nullptr);
        scalar_from_bytes(e[4].raw, sc + TAS_SC_TBF * 8, nullptr);
        scalar_from_bytes(e[5].raw, sc + TAS_SC_EQ * 8, nullptr);
        bool canon;
        scalar_from_bytes(e[6].raw, sc + TAS_SC_CHAL * 8, &canon);
        sa.chal_canonical = canon;
        for (size_t j = 0; j < ai.n_in; j++) {
          scalar_from_bytes(iv[j], sc + (TAS_SC_IV + j) * 8, nullptr);
          scalar_from_bytes(ibf[j], sc + (TAS_SC_IV + ai.n_in + j) * 8, nullptr);
        }
      }
    } else if (!e[0].present || !e[1].present || !e[2].present || !e[3].present) {
      panic = true;  // sametype.go:169-171 dereferences every field
    } else {
      scalar_from_bytes(e[0].raw, sc + ST_SC_TYPE * 8, nullptr);
      scalar_from_bytes(e[1].raw, sc + ST_SC_BF * 8, nullptr);
      bool canon;
      scalar_from_bytes(e[2].raw, sc + ST_SC_CHAL * 8, &canon);
      sa.chal_canonical = canon;
    }
    if (panic) return fail(FTS_E_MALFORMED);
    if (nil_fields) {
      // element arrays / CT must still decode even when the proof is rejected for nil fields
      G1A tmp;
      if (e[0].present && !g1_from_bytes(raw, 64, tmp)) return fail(FTS_E_MALFORMED);
      // the range proofs' slotted points too (the unslotted ones decoded above)
      for (int j = 0; j < s.rp_count && s.rp_base >= 0; j++)
        for (int q = 0; q < npts_rp; q++)
          if (q != RP_PT_V && !g1_from_bytes(hp + o_rraw + ((size_t)(s.rp_base + j) * npts_rp + q) * 64, 64, tmp))
            return fail(FTS_E_MALFORMED);
      return fail(FTS_E_TAS_INVALID);
    }
  };
  const double t_p2 = now_ms();
  // ---- 3. lay out and decode, chunk by chunk from its base
  parallel_for(nch, 2, [&](size_t q) {
    Run run = base[q];
    for (size_t i = q * CH; i < std::min(A, (q + 1) * CH); i++) decode_one(i, run);
  });
  const double t1 = now_ms();
  sl->parse_ms = (float)(t1 - t0);
  sl->phase_ms[0] = (float)(t_p1 - t0);
  sl->phase_ms[1] = (float)(t_p2 - t_p1);
  sl->phase_ms[2] = (float)(t1 - t_p2);
  // the slot's views: range-proof batch and sigma batch over the device copy
  uint8_t* dv = sl->dev;
  fts_rp_batch* b = sl->b;
  b->B = rp_total;
  b->raw = dv + o_rraw;
  b->sc = reinterpret_cast<uint32_t*>(dv + o_rsc);
  b->status0 = reinterpret_cast<int32_t*>(dv + o_rst);
  b->ipa_flag = reinterpret_cast<int32_t*>(dv + o_ripa);
  b->status = nullptr;  // never verified in place: the pass gathers it
  b->dense = false;     // action calls have no batch across calls (FTS_GT_ADAPT: groups of 256)
  b->locate_skip = c->act_locate_skip.load(std::memory_order_relaxed);  // the calls' shared backoff
  b->locate_backoff = c->act_locate_backoff.load(std::memory_order_relaxed);
  b->merged = 1;
  b->ntim = 0;
  sl->rp_res.assign((size_t)rp_total, FTS_E_NOT_RUN);
  sl->sig_res = reinterpret_cast<int32_t*>(hp + o_res);
  SigBatchDev& sd = sl->sd;
  sd = SigBatchDev{};
  sd.A = SA;
  sd.npts = pt_off;
  sd.naff = aff_off;
  sd.nwork = (int)nwork;
  sd.nfix = nfix_total;
  sd.act = reinterpret_cast<const SigAction*>(dv + o_act);
  sd.raw = dv + o_raw;
  sd.pt_owner = reinterpret_cast<int32_t*>(dv + o_owner);
  sd.pts = reinterpret_cast<uint32_t*>(dv + w_pts);
  sd.sc = reinterpret_cast<uint32_t*>(dv + o_sc);
  sd.status = reinterpret_cast<int32_t*>(dv + o_sst);
  sd.work = reinterpret_cast<int2*>(dv + o_work);
  sd.terms = reinterpret_cast<uint32_t*>(dv + w_terms);
  sd.aff = reinterpret_cast<uint32_t*>(dv + w_aff);
  sd.aff_off = reinterpret_cast<int32_t*>(dv + o_affoff);
  sd.msgs = dv + w_msgs;
  sd.jac = reinterpret_cast<uint32_t*>(dv + w_jac);
  sd.scratch = reinterpret_cast<uint32_t*>(dv + w_scratch);
  sd.rp_k = k;
  if ((SA || rp_total) && c->device >= 0) {
    // upload, then the sigma proofs at once on the slot's stream: decode + primes (and
    // the V slots of the call's own range proofs, before any pass gathers them), the
    // equations and transcripts.  No host wait: the pass waits for ev_sig[2], and the
    // pinned records stay the slot's until the call returns.
    sd.rp_raw = rp_total ? b->raw : nullptr;
    HIP_OK(hipMemcpyAsync(dv, hp, in_end, hipMemcpyHostToDevice, sl->s));
    HIP_OK(hipEventRecord(sl->ev_sig[0], sl->s));
    if (SA) launch_sig_prep(sd, sl->s);
    HIP_OK(hipEventRecord(sl->ev_sig[1], sl->s));
    if (SA) launch_sig_finish(sd, c->d_tables, c->n, sl->s);
    HIP_OK(hipEventRecord(sl->ev_sig[2], sl->s));
    HIP_OK(hipGetLastError());
  }
  sl->stage_ms = (float)(now_ms() - t1);
  return FTS_API_OK;
}

// Verify an action call: stage it, let the dispatcher verify it (alone or with
// other queued calls), then combine each action's sigma and range-proof verdicts
// with the reference's precedence.
static int act_verify(fts_ctx* c, const std::vector<ActionIn>& acts, int32_t* status, int32_t* fail_index) {
  ActSlot* sl = aslot_acquire(c);
  if (!sl) return FTS_API_ENOMEM;
  int rc = act_stage(c, sl, acts);
  if (rc == FTS_API_OK && sl->b->B) {
    RpReq me(sl->b, sl->rp_res.data(), sl);
    rc = rp_dispatch(c, me);
    c->act_locate_skip.store(sl->b->locate_skip, std::memory_order_relaxed);
    c->act_locate_backoff.store(sl->b->locate_backoff, std::memory_order_relaxed);
  } else if (rc == FTS_API_OK && sl->sd.A) {  // sigma proofs only (1-in/1-out transfers): no pass
    if (hipMemcpyAsync(sl->sig_res, sl->sd.status, (size_t)sl->sd.A * 4, hipMemcpyDeviceToHost, sl->s) != hipSuccess ||
        hipEventRecord(sl->done, sl->s) != hipSuccess || hipEventSynchronize(sl->done) != hipSuccess)
      rc = FTS_API_EDEVICE;
  }
  if (rc == FTS_API_OK) {
    const std::vector<ActionState>& st = sl->st;
    const int32_t* sig_res = sl->sig_res;
    const int32_t* rp_res = sl->rp_res.data();
    for (size_t i = 0; i < acts.size(); i++) {
      const ActionState& s = st[i];
      int32_t out = FTS_OK, idx = -1;
      if (s.host_final >= 0) {
        out = s.host_final;
      } else {
        const int32_t sig = sig_res[s.sig];
        bool malformed = sig == FTS_E_MALFORMED;
        for (int j = 0; j < s.rp_count && s.rp_base >= 0; j++) malformed |= rp_res[s.rp_base + j] == FTS_E_MALFORMED;
        if (malformed) {
          out = FTS_E_MALFORMED;                       // deserialisation precedes verification
        } else if (sig != FTS_OK) {
          out = sig;                                   // TypeAndSum / SameType error wins (transfer.go:192-196)
        } else if (s.rc_applicable) {
          if (s.rc_count_bad) {
            out = FTS_E_RC_COUNT;                      // rangecorrectness.go:138-140
          } else {
            for (int j = 0; j < s.rp_count; j++)       // first failing index wins (:141-160)
              if (rp_res[s.rp_base + j] != FTS_OK) {
                out = rp_res[s.rp_base + j];
                idx = j;
                break;
              }
          }
        }
      }
      status[i] = out;
      if (fail_index) fail_index[i] = idx;
    }
  }
  aslot_release(c, sl);
  return rc;
}

// host-side cost of act_stage (parse + layout, no device): tools/host_parse_bench.py
extern "C" int fts_debug_stage_actions(fts_ctx* c, size_t n_tr, const fts_transfer_item* transfers, size_t n_is,
                                       const fts_issue_item* issues, int reps, float* ms_avg) {
  if (!c || (n_tr && !transfers) || (n_is && !issues) || reps < 1 || c->device >= 0 || !c->shards.empty())
    return FTS_API_EINVAL;
  std::vector<ActionIn> acts;
  for (size_t i = 0; i < n_tr; i++)
    acts.push_back(ActionIn{SIG_TAS, transfers[i].inputs, transfers[i].n_in, transfers[i].outputs, transfers[i].n_out,
                            der::Span{transfers[i].proof, transfers[i].proof ? transfers[i].proof_len : 0}});
  for (size_t i = 0; i < n_is; i++)
    acts.push_back(ActionIn{SIG_ST, nullptr, 0, issues[i].tokens, issues[i].n_tok,
                            der::Span{issues[i].proof, issues[i].proof ? issues[i].proof_len : 0}});
  ActSlot sl;
  fts_rp_batch b;
  sl.b = &b;
  double tot[4] = {0, 0, 0, 0};
  if (int rc = act_stage(c, &sl, acts)) return rc;  // untimed: the slot's buffers grow (page faults) once
  for (int r = 0; r < reps; r++) {
    if (int rc = act_stage(c, &sl, acts)) return rc;
    tot[0] += sl.parse_ms;
    for (int q = 0; q < 3; q++) tot[1 + q] += sl.phase_ms[q];
  }
  sl.b = nullptr;
  if (ms_avg)
    for (int q = 0; q < 4; q++) ms_avg[q] = (float)(tot[q] / reps);
  return FTS_API_OK;
}


extern "C" {

int fts_transfer_verify_batch(fts_ctx* c, size_t n, const fts_transfer_item* items, int32_t* status,
                              int32_t* fail_index) {
  if (!c || !status || (n && !items)) return FTS_API_EINVAL;
  if (!c->shards.empty()) {
    std::vector<double> w(n);
    for (size_t i = 0; i < n; i++) w[i] = action_weight(items[i].n_in, items[i].n_out, true);
    return run_shards(plan(n, &w, (int)c->shards.size()), [&](int j, size_t lo, size_t hi) {
      return fts_transfer_verify_batch(c->shards[j], hi - lo, items + lo, status + lo,
                                       fail_index ? fail_index + lo : nullptr);
    });
  }
  if (c->device < 0) return FTS_API_EDEVICE;
  if (n == 0) return FTS_API_OK;
  std::vector<ActionIn> acts(n);
  for (size_t i = 0; i < n; i++)
    acts[i] = ActionIn{SIG_TAS, items[i].inputs, items[i].n_in, items[i].outputs, items[i].n_out,
                       der::Span{items[i].proof, items[i].proof ? items[i].proof_len : 0}};
  HIP_OK(hipSetDevice(c->device));
  int rc = act_verify(c, acts, status, fail_index);
  if (rc != FTS_API_OK)
    for (size_t i = 0; i < n; i++) status[i] = FTS_E_NOT_RUN;
  return rc;
}

int fts_issue_verify_batch(fts_ctx* c, size_t n, const fts_issue_item* items, int32_t* status, int32_t* fail_index) {
  if (!c || !status || (n && !items)) return FTS_API_EINVAL;
  if (!c->shards.empty()) {
    std::vector<double> w(n);
    for (size_t i = 0; i < n; i++) w[i] = action_weight(0, items[i].n_tok, false);
    return run_shards(plan(n, &w, (int)c->shards.size()), [&](int j, size_t lo, size_t hi) {
      return fts_issue_verify_batch(c->shards[j], hi - lo, items + lo, status + lo, fail_index ? fail_index + lo : nullptr);
    });
  }
  if (c->device < 0) return FTS_API_EDEVICE;
  if (n == 0) return FTS_API_OK;
  std::vector<ActionIn> acts(n);
  for (size_t i = 0; i < n; i++)
    acts[i] = ActionIn{SIG_ST, nullptr, 0, items[i].tokens, items[i].n_tok,
                       der::Span{items[i].proof, items[i].proof ? items[i].proof_len : 0}};
  HIP_OK(hipSetDevice(c->device));
  int rc = act_verify(c, acts, status, fail_index);
  if (rc != FTS_API_OK)
    for (size_t i = 0; i < n; i++) status[i] = FTS_E_NOT_RUN;
  return rc;
}

// mixed batch (BASELINE config C5): the transfers and issues of many token
// requests verified in ONE device pass (one range-proof batch + one sigma batch)
int fts_actions_verify_batch(fts_ctx* c, size_t n_tr, const fts_transfer_item* transfers, size_t n_is,
                             const fts_issue_item* issues, int32_t* status_tr, int32_t* fail_tr, int32_t* status_is,
                             int32_t* fail_is) {
  if (!c || (n_tr && (!transfers || !status_tr)) || (n_is && (!issues || !status_is))) return FTS_API_EINVAL;
  if (!c->shards.empty()) {  // transfers and issues each split into balanced shards, device j gets part j of both
    const int ns = (int)c->shards.size();
    std::vector<double> wt(n_tr), wi(n_is);
    for (size_t i = 0; i < n_tr; i++) wt[i] = action_weight(transfers[i].n_in, transfers[i].n_out, true);
    for (size_t i = 0; i < n_is; i++) wi[i] = action_weight(0, issues[i].n_tok, false);
    const std::vector<size_t> bt = plan(n_tr, &wt, ns), bi = plan(n_is, &wi, ns);
    std::vector<size_t> all(ns + 1);
    for (int j = 0; j <= ns; j++) all[j] = j;
    return run_shards(all, [&](int j, size_t, size_t) {
      const size_t t0 = bt[j], t1 = bt[j + 1], i0 = bi[j], i1 = bi[j + 1];
      if (t1 == t0 && i1 == i0) return FTS_API_OK;
      return fts_actions_verify_batch(c->shards[j], t1 - t0, transfers + t0, i1 - i0, issues + i0,
                                      status_tr ? status_tr + t0 : nullptr, fail_tr ? fail_tr + t0 : nullptr,
                                      status_is ? status_is + i0 : nullptr, fail_is ? fail_is + i0 : nullptr);
    });
  }
  if (c->device < 0) return FTS_API_EDEVICE;
  const size_t n = n_tr + n_is;
  if (n == 0) return FTS_API_OK;
  std::vector<ActionIn> acts(n);
  for (size_t i = 0; i < n_tr; i++)
    acts[i] = ActionIn{SIG_TAS, transfers[i].inputs, transfers[i].n_in, transfers[i].outputs, transfers[i].n_out,
                       der::Span{transfers[i].proof, transfers[i].proof ? transfers[i].proof_len : 0}};
  for (size_t i = 0; i < n_is; i++)
    acts[n_tr + i] = ActionIn{SIG_ST, nullptr, 0, issues[i].tokens, issues[i].n_tok,
                              der::Span{issues[i].proof, issues[i].proof ? issues[i].proof_len : 0}};
  std::vector<int32_t> st(n, FTS_E_NOT_RUN), fi(n, -1);
  HIP_OK(hipSetDevice(c->device));
  int rc;
  rc = act_verify(c, acts, st.data(), fi.data());
  if (rc != FTS_API_OK) std::fill(st.begin(), st.end(), FTS_E_NOT_RUN);
  for (size_t i = 0; i < n_tr; i++) {
    status_tr[i] = st[i];
    if (fail_tr) fail_tr[i] = fi[i];
  }
  for (size_t i = 0; i < n_is; i++) {
    status_is[i] = st[n_tr + i];
    if (fail_is) fail_is[i] = fi[n_tr + i];
  }
  return rc;
}

// Raw TokenRequest ingest: decode n requests on the host threads, verify the
// proofs of every action of every request in one device pass, then fold each
// request's action verdicts in the reference's order (issues, then transfers).
int fts_request_verify_batch(fts_ctx* c, size_t n, const uint8_t* const* req, const size_t* req_len,
                             int32_t* status, int32_t* fail_action, int32_t* fail_index) {
  if (!c || !status || (n && (!req || !req_len))) return FTS_API_EINVAL;
  if (!c->shards.empty()) {  // request bytes approximate the proofs they carry
    std::vector<double> w(n);
    for (size_t i = 0; i < n; i++) w[i] = (double)req_len[i] + 64.0;
    return run_shards(plan(n, &w, (int)c->shards.size()), [&](int j, size_t lo, size_t hi) {
      return fts_request_verify_batch(c->shards[j], hi - lo, req + lo, req_len + lo, status + lo,
                                      fail_action ? fail_action + lo : nullptr, fail_index ? fail_index + lo : nullptr);
    });
  }
  if (c->device < 0) return FTS_API_EDEVICE;
  if (n == 0) return FTS_API_OK;
  namespace rq = fts::host::req;
  std::vector<rq::Request> R(n);
  {
    unsigned nth = n >= 64 ? host_threads() : 1u;
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nth; t++)
      th.emplace_back([&]() {
        for (size_t i; (i = next++) < n;)
          rq::parse_request(req[i], req[i] ? req_len[i] : 0, SIG_TAS, SIG_ST, R[i]);
      });
    for (auto& t : th) t.join();
  }
  // actions that reach the verifier: those before (and excluding) the request's
  // first structurally invalid action
  std::vector<ActionIn> acts;
  std::vector<std::pair<uint32_t, uint32_t>> owner;  // (request, position in acts order)
  for (size_t i = 0; i < n; i++) {
    if (R[i].deser_failed) continue;
    for (size_t j = 0; j < R[i].acts.size(); j++) {
      const rq::Action& a = R[i].acts[j];
      if (a.pre >= 0) break;
      acts.push_back(ActionIn{a.kind, R[i].in(a), a.n_in, R[i].out(a), a.n_out, der::Span{a.proof, a.proof_len}});
      owner.emplace_back((uint32_t)i, (uint32_t)j);
    }
  }
  std::vector<int32_t> st(acts.size(), FTS_OK), fi(acts.size(), -1);
  int rc = FTS_API_OK;
  if (!acts.empty()) {
    HIP_OK(hipSetDevice(c->device));
    rc = act_verify(c, acts, st.data(), fi.data());
  }
  // fold: first failing verified action, else the first structural verdict
  std::vector<int32_t> first(n, -1);  // index into acts of the request's first failing action
  for (size_t q = acts.size(); q-- > 0;)
    if (st[q] != FTS_OK) first[owner[q].first] = (int32_t)q;
  for (size_t i = 0; i < n; i++) {
    const rq::Request& r = R[i];
    int32_t s = r.status, fa = r.fail_action, fx = -1;
    if (rc != FTS_API_OK) {
      s = FTS_E_NOT_RUN, fa = -1;
    } else if (!r.deser_failed) {
      if (first[i] >= 0) {
        const int q = first[i];
        s = st[q], fx = fi[q], fa = r.acts[owner[q].second].index;
      } else {
        for (const rq::Action& a : r.acts)
          if (a.pre >= 0) {
            s = a.pre, fa = a.index;
            break;
          }
      }
    }
    status[i] = s;
    if (fail_action) fail_action[i] = fa;
    if (fail_index) fail_index[i] = fx;
  }
  return rc;
}

int fts_request_inspect(const uint8_t* req, size_t req_len, int32_t* status, int32_t* fail_action, int32_t* n_issue,
                        int32_t* n_transfer, int32_t* pre_status, int32_t* pre_action) {
  if (!status || (req_len && !req)) return FTS_API_EINVAL;
  fts::host::req::Request r;
  fts::host::req::parse_request(req, req ? req_len : 0, SIG_TAS, SIG_ST, r);
  int32_t ni = 0, nt = 0, ps = FTS_OK, pa = -1;
  for (const auto& a : r.acts) {
    (a.transfer ? nt : ni)++;
    if (a.pre >= 0 && pa < 0) ps = a.pre, pa = a.index;
  }
  *status = r.status;
  if (fail_action) *fail_action = r.fail_action;
  if (n_issue) *n_issue = ni;
  if (n_transfer) *n_transfer = nt;
  if (pre_status) *pre_status = ps;
  if (pre_action) *pre_action = pa;
  return FTS_API_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ prover
namespace fts {
namespace host {
RngSource::RngSource(uint64_t sd) : secure(sd == FTS_SEED_OS_RANDOM), seed(sd) {
  if (secure) ok = getrandom(key, sizeof key, 0) == (ssize_t)sizeof key;
}
}  // namespace host
}  // namespace fts

static const ProverTables& prover_tables(const fts_ctx* cc) {
  fts_ctx* c = const_cast<fts_ctx*>(cc);
  std::call_once(c->prover_once, [&]() { build_prover_tables(c->pp, c->n, c->ptab); });
  return c->ptab;
}

static bool fr_arg(const uint8_t* b32, Fr& out) {
  if (!b32) return false;
  out = fr_from_be(b32);
  return true;
}

int fts_token_commit(const fts_ctx* c, const uint8_t* type, size_t type_len, uint64_t value, const uint8_t* bf32,
                     uint8_t* com64_out) {
  Fr bf;
  if (!c || !com64_out || !fr_arg(bf32, bf)) return FTS_API_EINVAL;
  const ProverTables& T = prover_tables(c);
  G1A t = token_commit(T, type_to_zr(type, type_len), value, bf);
  g1_to_bytes(t, com64_out);
  return FTS_API_OK;
}

int fts_rp_prove(const fts_ctx* c, uint64_t value, const uint8_t* bf32, uint64_t seed, uint8_t* out_der,
                 size_t out_cap, size_t* out_len, uint8_t* com64_out) {
  Fr bf;
  if (!c || !out_der || !out_len || !fr_arg(bf32, bf)) return FTS_API_EINVAL;
  const ProverTables& T = prover_tables(c);
  Msm vm;
  vm.add_fb(T.ped(1), fr_u64(value));
  vm.add_fb(T.ped(2), bf);
  G1A V = vm.aff();
  RngSource src(seed);
  if (!src.ok) return FTS_API_EDEVICE;
  Rng rng = src.at(0);
  RangeProofOut rp = prove_range(T, c->pp, c->n, c->k, V, value, bf, rng);
  std::string s = rp.serialize();
  *out_len = s.size();
  if (s.size() > out_cap) return FTS_API_ESIZE;
  memcpy(out_der, s.data(), s.size());
  if (com64_out) g1_to_bytes(V, com64_out);
  return FTS_API_OK;
}

int fts_rp_prove_batch(const fts_ctx* c, size_t n, const uint64_t* values, const uint8_t* bfs, uint64_t seed,
                       int threads, uint8_t* out, size_t out_cap, size_t* offsets, size_t* lens,
                       uint8_t* com64_out) {
  if (!c || !values || !bfs || !out || !offsets || !lens || !com64_out) return FTS_API_EINVAL;
  const ProverTables& T = prover_tables(c);
  RngSource src(seed);
  if (!src.ok) return FTS_API_EDEVICE;
  std::vector<std::string> res(n);
  std::atomic<size_t> next{0};
  int nth = threads > 0 ? threads : (int)host_threads();
  std::vector<std::thread> th;
  for (int t = 0; t < nth; t++)
    th.emplace_back([&]() {
      for (size_t i; (i = next++) < n;) {
        Fr bf = fr_from_be(bfs + 32 * i);
        Msm vm;
        vm.add_fb(T.ped(1), fr_u64(values[i]));
        vm.add_fb(T.ped(2), bf);
        G1A V = vm.aff();
        Rng rng = src.at(i);
        res[i] = prove_range(T, c->pp, c->n, c->k, V, values[i], bf, rng).serialize();
        g1_to_bytes(V, com64_out + 64 * i);
      }
    });
  for (auto& t : th) t.join();
  size_t off = 0;
  for (size_t i = 0; i < n; i++) {
    if (off + res[i].size() > out_cap) return FTS_API_ESIZE;
    memcpy(out + off, res[i].data(), res[i].size());
    offsets[i] = off;
    lens[i] = res[i].size();
    off += res[i].size();
  }
  return FTS_API_OK;
}

int fts_transfer_prove(const fts_ctx* c, const uint8_t* type, size_t type_len, size_t n_in, const uint64_t* in_values,
                       const uint8_t* in_bfs, size_t n_out, const uint64_t* out_values, const uint8_t* out_bfs,
                       uint64_t seed, uint8_t* out_der, size_t out_cap, size_t* out_len) {
  if (!c || !out_der || !out_len || !n_in || !n_out) return FTS_API_EINVAL;
  const ProverTables& T = prover_tables(c);
  std::vector<uint64_t> iv(in_values, in_values + n_in), ov(out_values, out_values + n_out);
  std::vector<Fr> ib(n_in), ob(n_out);
  for (size_t i = 0; i < n_in; i++) ib[i] = fr_from_be(in_bfs + 32 * i);
  for (size_t i = 0; i < n_out; i++) ob[i] = fr_from_be(out_bfs + 32 * i);
  RngSource src(seed);
  if (!src.ok) return FTS_API_EDEVICE;
  Rng rng = src.at(0);
  std::string s = prove_transfer(T, c->pp, c->n, c->k, type_to_zr(type, type_len), iv, ib, ov, ob, rng);
  *out_len = s.size();
  if (s.size() > out_cap) return FTS_API_ESIZE;
  memcpy(out_der, s.data(), s.size());
  return FTS_API_OK;
}

int fts_issue_prove(const fts_ctx* c, const uint8_t* type, size_t type_len, size_t n_tok, const uint64_t* values,
                    const uint8_t* bfs, uint64_t seed, uint8_t* out_der, size_t out_cap, size_t* out_len) {
  if (!c || !out_der || !out_len || !n_tok) return FTS_API_EINVAL;
  const ProverTables& T = prover_tables(c);
  std::vector<uint64_t> v(values, values + n_tok);
  std::vector<Fr> b(n_tok);
  for (size_t i = 0; i < n_tok; i++) b[i] = fr_from_be(bfs + 32 * i);
  RngSource src(seed);
  if (!src.ok) return FTS_API_EDEVICE;
  Rng rng = src.at(0);
  std::string s = prove_issue(T, c->pp, c->n, c->k, type_to_zr(type, type_len), v, b, rng);
  *out_len = s.size();
  if (s.size() > out_cap) return FTS_API_ESIZE;
  memcpy(out_der, s.data(), s.size());
  return FTS_API_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Token opening checks (crypto/audit/auditor.go:226-238, crypto/token/token.go:69-83)
// ---------------------------------------------------------------------------
namespace {
// canonical LE u32 limbs of a BE 32-byte integer reduced mod r (G1.Mul(s) = (s mod r) P)
void zr_canon_words(const uint8_t* be32, uint32_t out[8]) {
  uint64_t c[4];
  be32_to_u64(be32, c);
  while (geq_mod<ModR>(c)) sub_mod_raw<ModR>(c);
  for (int i = 0; i < 4; i++) out[2 * i] = (uint32_t)c[i], out[2 * i + 1] = (uint32_t)(c[i] >> 32);
}
void fr_canon_words(const Fr& a, uint32_t out[8]) {
  uint64_t c[4];
  from_mont(a, c);
  for (int i = 0; i < 4; i++) out[2 * i] = (uint32_t)c[i], out[2 * i + 1] = (uint32_t)(c[i] >> 32);
}
constexpr size_t OPEN_REC = 64 + 96 + 4;       // staged bytes per token
constexpr double OPEN_PRODUCTS = 48.0 * 11 + 4;  // Fp products: <= 48 mixed additions + the projective compare
}  // namespace

extern "C" {

int fts_token_open_batch(fts_ctx* c, size_t n, const fts_token_opening* items, int32_t* status) {
  if (!c || n > (size_t)(1u << 26) || (n && (!items || !status))) return FTS_API_EINVAL;
  if (n == 0) return FTS_API_OK;
  if (!c->shards.empty())
    return run_shards(plan(n, nullptr, (int)c->shards.size()), [&](int j, size_t lo, size_t hi) {
      return fts_token_open_batch(c->shards[j], hi - lo, items + lo, status + lo);
    });
  if (c->device < 0) return FTS_API_EDEVICE;
  HIP_OK(hipSetDevice(c->device));
  LaneGuard lg(c);
  Lane& L = *lg.L;
  const double t0 = now_ms();
  uint8_t* st = L.stage_buf(n * OPEN_REC);
  if (!st || L.ws.open_rec.ensure(n * OPEN_REC)) return FTS_API_ENOMEM;
  uint8_t* h_raw = st;
  uint32_t* h_sc = reinterpret_cast<uint32_t*>(st + n * 64);
  int32_t* h_st = reinterpret_cast<int32_t*>(st + n * 160);
  // host: HashToZr(type) (one SHA-256 per distinct type within a chunk), scalars mod r
  const size_t CH = 512, nch = (n + CH - 1) / CH;
  parallel_for(nch, 2, [&](size_t ch) {
    // HashToZr of the last few distinct types (a batch carries few token types)
    constexpr int NC = 8;
    std::string key[NC];
    uint32_t val[NC][8];
    int nc = 0, rr = 0;
    for (size_t i = ch * CH; i < std::min(n, (ch + 1) * CH); i++) {
      const fts_token_opening& it = items[i];
      uint32_t* S = h_sc + i * 24;
      if (!it.com64 || !it.value32 || !it.bf32 || (it.type_len && !it.type)) {
        h_st[i] = FTS_E_MALFORMED;
        memset(h_raw + i * 64, 0, 64);
        memset(S, 0, 96);
        continue;
      }
      h_st[i] = FTS_OK;
      memcpy(h_raw + i * 64, it.com64, 64);
      int hit = -1;
      for (int q = 0; q < nc && hit < 0; q++)
        if (key[q].size() == it.type_len && !memcmp(key[q].data(), it.type, it.type_len)) hit = q;
      if (hit < 0) {
        hit = nc < NC ? nc++ : (rr++ % NC);
        key[hit].assign((const char*)it.type, it.type_len);
        fr_canon_words(hash_to_zr(key[hit]), val[hit]);
      }
      memcpy(S, val[hit], 32);
      zr_canon_words(it.value32, S + 8);
      zr_canon_words(it.bf32, S + 16);
    }
  });
  const double t1 = now_ms();
  uint8_t* d = L.ws.open_rec.as<uint8_t>();
  L.tl.begin(L.s);
  HIP_OK(hipMemcpyAsync(d, st, n * OPEN_REC, hipMemcpyHostToDevice, L.s));
  L.tl.mark("h2d_open", L.s, 0);
  launch_open_check((int)n, d, reinterpret_cast<const uint32_t*>(d + n * 64), c->d_tables, c->n,
                    reinterpret_cast<int32_t*>(d + n * 160), L.s);
  L.tl.mark("k_open_check", L.s, OPEN_PRODUCTS * (double)n);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(h_st, d + n * 160, n * 4, hipMemcpyDeviceToHost, L.s));
  const double t2 = now_ms();
  HIP_OK(L.sync());
  memcpy(status, h_st, n * 4);
  L.host_parse_ms = (float)(t1 - t0);
  L.host_stage_ms = 0;
  L.host_prep_ms = 0;
  L.host_enqueue_ms = (float)(t2 - t1);
  L.host_wait_ms = (float)(now_ms() - t2);
  collect_timings(c, L, nullptr);
  return FTS_API_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Batched range-proof prover on the device (prove_kernels.hip)
// ---------------------------------------------------------------------------
namespace {
constexpr size_t PV_CHUNK = 16384;  // proofs per device pass (~54 KB of arena each at n = 64)

struct PvArena {
  size_t off = 0;
  template <class T>
  size_t take(size_t count) {
    size_t o = off;
    off += (count * sizeof(T) + 255) & ~(size_t)255;
    return o;
  }
};

// stage tables: per-term table slot, groups {t0, t1, seg} of <= PV_TPG terms, segments {g0, g1}
struct PvStageHost {
  std::vector<int32_t> base;
  std::vector<int32_t> grp;  // 4 per group
  std::vector<int32_t> seg;  // 2 per segment
  void segment(int t0, int t1) {  // terms [t0, t1) form the next output point
    const int s = (int)seg.size() / 2, g0 = (int)grp.size() / 4;
    for (int t = t0; t < t1; t += PV_TPG) grp.insert(grp.end(), {t, std::min(t1, t + PV_TPG), s, 0});
    seg.insert(seg.end(), {g0, (int)grp.size() / 4});
  }
};

std::vector<PvStageHost> pv_stage_tables(int n, int k) {
  std::vector<PvStageHost> st(3 + k);
  PvStageHost& s1 = st[0];  // V | C (rho P) | D
  s1.base = {tb_G(n), tb_H(n), tb_P(n)};
  for (int i = 0; i < n; i++) s1.base.insert(s1.base.end(), {i, n + i});
  s1.base.push_back(tb_P(n));
  s1.segment(0, 2);
  s1.segment(2, 3);
  s1.segment(3, 2 * n + 4);
  PvStageHost& s2 = st[1];  // T1 | T2
  s2.base = {tb_G(n), tb_H(n), tb_G(n), tb_H(n)};
  s2.segment(0, 2);
  s2.segment(2, 4);
  PvStageHost& s3 = st[2];  // H'_0 | ... | H'_{n-1} | com
  for (int i = 0; i < n; i++) s3.base.push_back(n + i);
  for (int i = 0; i < n; i++) s3.base.insert(s3.base.end(), {i, n + i});
  for (int i = 0; i < n; i++) s3.segment(i, i + 1);
  s3.segment(n, 3 * n);
  for (int j = 0; j < k; j++) {  // L_j | R_j
    PvStageHost& r = st[3 + j];
    const int m = n >> (j + 1);
    for (int t = 0; t < n; t++) r.base.push_back((t % (2 * m)) >= m ? t : n + t);
    r.base.push_back(tb_Q(n));
    for (int t = 0; t < n; t++) r.base.push_back((t % (2 * m)) < m ? t : n + t);
    r.base.push_back(tb_Q(n));
    r.segment(0, n + 1);
    r.segment(n + 1, 2 * n + 2);
  }
  return st;
}
}  // namespace

// N range proofs on the device: input(i, value, bf8, rnd) supplies proof i's value, its
// blinding factor and its 2n + 4 random scalars (canonical limbs, pv_nrnd order);
// der[i] <- the serialized proof, com64_out[i] (optional) <- V
using PvInput = std::function<void(size_t, uint64_t&, uint32_t*, uint32_t*)>;
static int rp_prove_device(fts_ctx* c, Lane& L, size_t N, const PvInput& input, std::vector<std::string>& der,
                           uint8_t* com64_out) {
  const int n = c->n, k = c->k;
  // stage tables (proof-independent), uploaded once per call
  const std::vector<PvStageHost> sth = pv_stage_tables(n, k);
  std::vector<int32_t> tab;
  std::vector<size_t> tb_off;
  for (const PvStageHost& s : sth)
    for (const std::vector<int32_t>* v : {&s.base, &s.grp, &s.seg}) {
      while (tab.size() % 4) tab.push_back(0);  // int4 alignment of the group arrays
      tb_off.push_back(tab.size());
      tab.insert(tab.end(), v->begin(), v->end());
    }
  const size_t B0 = std::min(N, PV_CHUNK);
  PvArena ar;
  const size_t o_tab = ar.take<int32_t>(tab.size()), o_val = ar.take<uint64_t>(B0),
               o_rnd = ar.take<uint32_t>(B0 * pv_nrnd(n) * 8), o_bf = ar.take<uint32_t>(B0 * 8),
               o_st = ar.take<uint32_t>(B0 * pv_nst(n) * 8), o_terms = ar.take<uint32_t>(B0 * pv_tmax(n) * 8),
               o_part = ar.take<uint32_t>(B0 * pv_gmax(n) * 24), o_jac = ar.take<uint32_t>(B0 * (n + 1) * 24),
               o_aff = ar.take<uint32_t>(B0 * (n + 1) * 16), o_hp = ar.take<uint8_t>(B0 * (n + 1) * 64),
               o_out = ar.take<uint8_t>(B0 * pv_npts(k) * 64), o_fr = ar.take<uint32_t>(B0 * PV_NFR * 8),
               o_ch = ar.take<uint32_t>(B0 * rp_nch(k) * 8), o_sc = ar.take<uint32_t>(B0 * RP_NSC * 8),
               o_status = ar.take<int32_t>(B0), o_x0 = ar.take<uint8_t>(B0 * x0_var_bytes(n)),
               o_hs = ar.take<uint8_t>(B0 * PV_HSLOT);
  if (L.ws.pv.ensure(ar.off)) return FTS_API_ENOMEM;
  uint8_t* base = L.ws.pv.as<uint8_t>();
  // pinned staging: inputs [values | rnd | bf], outputs [points | scalars]
  const size_t in_bytes = B0 * (8 + pv_nrnd(n) * 32 + 32), out_pts_b = B0 * pv_npts(k) * 64,
               out_fr_b = B0 * PV_NFR * 32;
  uint8_t* stg = L.stage_buf(in_bytes + out_pts_b + out_fr_b);
  if (!stg) return FTS_API_ENOMEM;
  HIP_OK(hipMemcpyAsync(base + o_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, L.s));
  HIP_OK(hipMemsetAsync(base + o_status, 0, B0 * 4, L.s));
  PvStage stages[3 + 16];
  for (size_t s = 0; s < sth.size(); s++) {
    const int32_t* tb = reinterpret_cast<const int32_t*>(base + o_tab);
    stages[s].T = (int)sth[s].base.size();
    stages[s].G = (int)sth[s].grp.size() / 4;
    stages[s].S = (int)sth[s].seg.size() / 2;
    stages[s].base = tb + tb_off[3 * s];
    stages[s].grp = reinterpret_cast<const int4*>(tb + tb_off[3 * s + 1]);
    stages[s].seg = reinterpret_cast<const int2*>(tb + tb_off[3 * s + 2]);
  }
  der.assign(N, std::string());
  for (size_t p0 = 0; p0 < N; p0 += B0) {
    const size_t B = std::min(B0, N - p0);
    uint64_t* h_val = reinterpret_cast<uint64_t*>(stg);
    uint32_t* h_rnd = reinterpret_cast<uint32_t*>(stg + B0 * 8);
    uint32_t* h_bf = reinterpret_cast<uint32_t*>(stg + B0 * 8 + B0 * pv_nrnd(n) * 32);
    // randomness in the host prover's draw order (prove_range): rho, eta, (rl_i, rr_i), tau1, tau2
    const double h0 = now_ms();
    parallel_for(B, 256, [&](size_t i) { input(p0 + i, h_val[i], h_bf + i * 8, h_rnd + i * pv_nrnd(n) * 8); });
    HIP_OK(hipMemcpyAsync(base + o_val, h_val, B * 8, hipMemcpyHostToDevice, L.s));
    HIP_OK(hipMemcpyAsync(base + o_rnd, h_rnd, B * pv_nrnd(n) * 32, hipMemcpyHostToDevice, L.s));
    HIP_OK(hipMemcpyAsync(base + o_bf, h_bf, B * 32, hipMemcpyHostToDevice, L.s));
    PvDev d;
    d.B = (int)B, d.n = n, d.k = k;
    d.tables = c->d_tables;
    d.values = reinterpret_cast<const uint64_t*>(base + o_val);
    d.rnd = reinterpret_cast<const uint32_t*>(base + o_rnd);
    d.bf = reinterpret_cast<const uint32_t*>(base + o_bf);
    d.st = reinterpret_cast<uint32_t*>(base + o_st);
    d.terms = reinterpret_cast<uint32_t*>(base + o_terms);
    d.partial = reinterpret_cast<uint32_t*>(base + o_part);
    d.jac = reinterpret_cast<uint32_t*>(base + o_jac);
    d.aff = reinterpret_cast<uint32_t*>(base + o_aff);
    d.hp_be = base + o_hp;
    d.out_pts = base + o_out;
    d.out_fr = reinterpret_cast<uint32_t*>(base + o_fr);
    d.ch = reinterpret_cast<uint32_t*>(base + o_ch);
    d.sc_ip = reinterpret_cast<uint32_t*>(base + o_sc);
    d.status = reinterpret_cast<int32_t*>(base + o_status);
    d.x0_msgs = base + o_x0;
    d.hslot = base + o_hs;
    const double h1 = now_ms();
    L.tl.begin(L.s);
    launch_rp_prove(d, stages, c->d_x0const, c->d_x0tmpl, L.s, &L.tl);
    HIP_OK(hipGetLastError());
    uint8_t* h_pts = stg + in_bytes;
    uint32_t* h_fr = reinterpret_cast<uint32_t*>(stg + in_bytes + out_pts_b);
    HIP_OK(hipMemcpyAsync(h_pts, base + o_out, B * pv_npts(k) * 64, hipMemcpyDeviceToHost, L.s));
    HIP_OK(hipMemcpyAsync(h_fr, base + o_fr, B * PV_NFR * 32, hipMemcpyDeviceToHost, L.s));
    const double h2 = now_ms();
    HIP_OK(L.sync());
    const double h3 = now_ms();
    bool bad = false;
    parallel_for(B, 256, [&](size_t i) {
      const uint8_t* P = h_pts + i * pv_npts(k) * 64;
      const uint32_t* F = h_fr + i * PV_NFR * 8;
      auto pt = [&](int slot) {
        G1A a;
        if (!g1_from_bytes(P + slot * 64, 64, a)) bad = true;
        return a;
      };
      auto fr = [&](int slot) {
        uint64_t w[4];
        for (int q = 0; q < 4; q++) w[q] = (uint64_t)F[slot * 8 + 2 * q] | ((uint64_t)F[slot * 8 + 2 * q + 1] << 32);
        return to_mont<ModR>(w);
      };
      RangeProofOut ro;
      ro.T1 = pt(PV_T1), ro.T2 = pt(PV_T2), ro.C = pt(PV_C), ro.D = pt(PV_D);
      ro.tau = fr(PV_F_TAU), ro.delta = fr(PV_F_DELTA), ro.ip = fr(PV_F_IP), ro.a = fr(PV_F_A), ro.b = fr(PV_F_B);
      for (int j = 0; j < k; j++) {
        ro.L.push_back(pt(PV_L(j)));
        ro.R.push_back(pt(PV_R(j)));
      }
      der[p0 + i] = ro.serialize();
      if (com64_out) memcpy(com64_out + 64 * (p0 + i), P + PV_V * 64, 64);
    });
    if (bad) return FTS_API_EDEVICE;  // a device point failed its own encoding check
    L.host_prep_ms = (float)(h1 - h0);         // randomness draw
    L.host_enqueue_ms = (float)(h2 - h1);
    L.host_wait_ms = (float)(h3 - h2);         // device
    L.host_parse_ms = (float)(now_ms() - h3);  // DER serialisation
    L.host_stage_ms = 0;
    collect_timings(c, L, nullptr);
  }
  return FTS_API_OK;
}

extern "C" {

int fts_rp_prove_batch_gpu(fts_ctx* c, size_t N, const uint64_t* values, const uint8_t* bfs, uint64_t seed,
                           uint8_t* out, size_t out_cap, size_t* offsets, size_t* lens, uint8_t* com64_out) {
  if (!c || !values || !bfs || !out || !offsets || !lens || !com64_out || N > (size_t)(1u << 24))
    return FTS_API_EINVAL;
  if (N == 0) return FTS_API_OK;
  if (!c->shards.empty())  // provers run on the first device of a multi-device context
    return fts_rp_prove_batch_gpu(c->shards[0], N, values, bfs, seed, out, out_cap, offsets, lens, com64_out);
  if (c->device < 0) return FTS_API_EDEVICE;
  HIP_OK(hipSetDevice(c->device));
  RngSource src(seed);
  if (!src.ok) return FTS_API_EDEVICE;
  LaneGuard lg(c);
  const int nr = pv_nrnd(c->n);
  std::vector<std::string> der;
  int rc = rp_prove_device(c, *lg.L, N, [&](size_t g, uint64_t& v, uint32_t* bf8, uint32_t* R) {
    v = values[g];
    Rng rng = src.at(g);  // the host prover's draw order (prove_range)
    for (int r = 0; r < nr; r++) fr_canon_words(rng.fr(), R + r * 8);
    fr_canon_words(fr_from_be(bfs + 32 * g), bf8);
  }, der, com64_out);
  if (rc) return rc;
  size_t off = 0;
  for (size_t i = 0; i < N; i++) {
    offsets[i] = off;
    lens[i] = der[i].size();
    if (off + der[i].size() > out_cap) return FTS_API_ESIZE;
    memcpy(out + off, der[i].data(), der[i].size());
    off += der[i].size();
  }
  return FTS_API_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Whole transfer / issue proofs on the device: sigma prover (k_sp_prove) + the
// range proofs of every output (rp_prove_device), byte-identical to
// fts_transfer_prove / fts_issue_prove for the same seeds
// ---------------------------------------------------------------------------
static int actions_prove_device(fts_ctx* c, size_t A, const fts_action_witness* w, int issue, uint64_t seed,
                                uint8_t* out, size_t out_cap, size_t* offsets, size_t* lens) {
  if (!c || !w || !out || !offsets || !lens || A > (size_t)(1u << 22)) return FTS_API_EINVAL;
  if (A == 0) return FTS_API_OK;
  if (c->device < 0) return FTS_API_EDEVICE;
  const int n = c->n, nr = pv_nrnd(n), kind = issue ? 1 : 0;
  for (size_t a = 0; a < A; a++) {
    const fts_action_witness& x = w[a];
    const size_t nin = issue ? 0 : x.n_in;
    if ((!issue && (!nin || !x.in_values || !x.in_bfs)) || !x.n_out || !x.out_values || !x.out_bfs ||
        (x.type_len && !x.type) || nin > 4096 || x.n_out > 4096)
      return FTS_API_EINVAL;
  }
  RngSource src(seed);
  if (!src.ok) return FTS_API_EDEVICE;
  HIP_OK(hipSetDevice(c->device));
  LaneGuard lg(c);
  Lane& L = *lg.L;
  // layout: offsets of every action's scalars / points / transcript / outputs / range proofs
  std::vector<SpAction> act(A);
  std::vector<size_t> rp_first(A + 1, 0);
  size_t nsc = 0, npt = 0, nmsg = 0, nout = 0;
  for (size_t a = 0; a < A; a++) {
    const int nin = issue ? 0 : (int)w[a].n_in, no = (int)w[a].n_out;
    const int m = sp_npts(kind, nin, no);
    act[a] = SpAction{kind, nin, no, (int32_t)nsc, (int32_t)npt, (int32_t)nmsg, (int32_t)nout,
                      kind == 0 ? 2 * nin + no + 2 : 0};
    nsc += sp_nsc(kind, nin, no);
    npt += m;
    nmsg += sp_msg_slot(m);
    nout += sp_nout(kind, nin);
    const bool has_rc = issue || nin != 1 || no != 1;  // transfer.go:85-87 (1-in/1-out: no range proof)
    rp_first[a + 1] = rp_first[a] + (has_rc ? no : 0);
  }
  const size_t NR = rp_first[A];
  std::vector<uint32_t> h_sc(nsc * 8);
  std::vector<uint64_t> rp_val(NR);
  std::vector<uint32_t> rp_bf(NR * 8), rp_rnd(NR * nr * 8);
  // host: the draws of the host prover, in its order (prove_transfer / prove_issue)
  parallel_for(A, 64, [&](size_t a) {
    const fts_action_witness& x = w[a];
    const SpAction& ac = act[a];
    uint32_t* S = h_sc.data() + (size_t)ac.sc_off * 8;
    Rng rng = src.at(a);
    const Fr type = type_to_zr(x.type, x.type_len);
    const Fr tbf = rng.fr();
    fr_canon_words(type, S);
    fr_canon_words(tbf, S + 8);
    auto rp_draw = [&](size_t q, uint64_t v, const uint8_t* bf32) {
      const size_t r = rp_first[a] + q;
      rp_val[r] = v;
      fr_canon_words(sub(fr_from_be(bf32), tbf), rp_bf.data() + r * 8);  // V = Out - CT
      for (int t = 0; t < nr; t++) fr_canon_words(rng.fr(), rp_rnd.data() + (r * nr + t) * 8);
    };
    const int N = ac.n_in, M = ac.n_out;
    if (!issue) {
      if (rp_first[a + 1] > rp_first[a])
        for (int j = 0; j < M; j++) rp_draw(j, x.out_values[j], x.out_bfs + 32 * j);
      fr_canon_words(rng.fr(), S + 2 * 8);  // r_t
      fr_canon_words(rng.fr(), S + 3 * 8);  // r_tbf
      for (int i = 0; i < N; i++) {
        fr_canon_words(rng.fr(), S + (5 + 2 * N + i) * 8);  // r_iv_i
        fr_canon_words(rng.fr(), S + (5 + 3 * N + i) * 8);  // r_ibf_i
      }
      fr_canon_words(rng.fr(), S + 4 * 8);  // r_sum
      for (int i = 0; i < N; i++) {
        fr_canon_words(fr_u64(x.in_values[i]), S + (5 + i) * 8);
        fr_canon_words(fr_from_be(x.in_bfs + 32 * i), S + (5 + N + i) * 8);
      }
      for (int j = 0; j < M; j++) {
        fr_canon_words(fr_u64(x.out_values[j]), S + (5 + 4 * N + j) * 8);
        fr_canon_words(fr_from_be(x.out_bfs + 32 * j), S + (5 + 4 * N + M + j) * 8);
      }
    } else {
      fr_canon_words(rng.fr(), S + 2 * 8);  // r_t
      fr_canon_words(rng.fr(), S + 3 * 8);  // r_bf
      for (int j = 0; j < M; j++) rp_draw(j, x.out_values[j], x.out_bfs + 32 * j);
    }
  });
  // device: sigma proofs
  PvArena ar;
  const size_t o_act = ar.take<SpAction>(A), o_sc = ar.take<uint32_t>(nsc * 8), o_jac = ar.take<uint32_t>(npt * 24),
               o_aff = ar.take<uint32_t>(npt * 16), o_be = ar.take<uint8_t>(npt * 64), o_msg = ar.take<uint8_t>(nmsg),
               o_out = ar.take<uint32_t>(nout * 8);
  if (L.ws.sp.ensure(ar.off)) return FTS_API_ENOMEM;
  uint8_t* base = L.ws.sp.as<uint8_t>();
  std::vector<uint8_t> h_be(npt * 64);
  std::vector<uint32_t> h_out(nout * 8);
  HIP_OK(hipMemcpyAsync(base + o_act, act.data(), A * sizeof(SpAction), hipMemcpyHostToDevice, L.s));
  HIP_OK(hipMemcpyAsync(base + o_sc, h_sc.data(), nsc * 32, hipMemcpyHostToDevice, L.s));
  SpDev d;
  d.A = (int)A, d.tables = c->d_tables, d.n = n;
  d.act = reinterpret_cast<const SpAction*>(base + o_act);
  d.sc = reinterpret_cast<const uint32_t*>(base + o_sc);
  d.jac = reinterpret_cast<uint32_t*>(base + o_jac);
  d.aff = reinterpret_cast<uint32_t*>(base + o_aff);
  d.be = base + o_be;
  d.msgs = base + o_msg;
  d.out = reinterpret_cast<uint32_t*>(base + o_out);
  launch_sigma_prove(d, L.s);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(h_be.data(), base + o_be, npt * 64, hipMemcpyDeviceToHost, L.s));
  HIP_OK(hipMemcpyAsync(h_out.data(), base + o_out, nout * 32, hipMemcpyDeviceToHost, L.s));
  HIP_OK(L.sync());
  // device: every range proof of the batch
  std::vector<std::string> rps;
  if (NR) {
    int rc = rp_prove_device(c, L, NR, [&](size_t r, uint64_t& v, uint32_t* bf8, uint32_t* R) {
      v = rp_val[r];
      memcpy(bf8, rp_bf.data() + r * 8, 32);
      memcpy(R, rp_rnd.data() + r * nr * 8, (size_t)nr * 32);
    }, rps, nullptr);
    if (rc) return rc;
  }
  // host: DER (transfer.go:140-149 / issue/prover.go:100-111)
  std::vector<std::string> der(A);
  bool bad = false;
  parallel_for(A, 64, [&](size_t a) {
    const SpAction& ac = act[a];
    const uint32_t* O = h_out.data() + (size_t)ac.out_off * 8;
    auto fr = [&](int i) {
      uint64_t q[4];
      for (int t = 0; t < 4; t++) q[t] = (uint64_t)O[i * 8 + 2 * t] | ((uint64_t)O[i * 8 + 2 * t + 1] << 32);
      return to_mont<ModR>(q);
    };
    G1A ct;
    if (!g1_from_bytes(h_be.data() + ((size_t)ac.pt_off + ac.ct_idx) * 64, 64, ct)) bad = true;
    std::vector<std::string> proofs;
    for (size_t r = rp_first[a]; r < rp_first[a + 1]; r++) proofs.push_back(rps[r]);
    if (!issue) {
      const int N = ac.n_in;
      std::vector<Fr> pibf(N), piv(N);
      for (int i = 0; i < N; i++) pibf[i] = fr(i), piv[i] = fr(N + i);
      std::string tas = der::values({el_g1(ct), el_fr_array(pibf), el_fr_array(piv), el_fr(fr(2 * N)),
                                     el_fr(fr(2 * N + 1)), el_fr(fr(2 * N + 2)), el_fr(fr(2 * N + 3))});
      der[a] = der::values({tas, proofs.empty() ? std::string() : rc_serialize(proofs)});
    } else {
      std::string st = der::values({el_fr(fr(0)), el_fr(fr(1)), el_fr(fr(2)), el_g1(ct)});
      der[a] = der::values({st, rc_serialize(proofs)});
    }
  });
  if (bad) return FTS_API_EDEVICE;
  size_t off = 0;
  for (size_t a = 0; a < A; a++) {
    offsets[a] = off;
    lens[a] = der[a].size();
    if (off + der[a].size() > out_cap) return FTS_API_ESIZE;
    memcpy(out + off, der[a].data(), der[a].size());
    off += der[a].size();
  }
  return FTS_API_OK;
}

extern "C" {
int fts_transfer_prove_batch_gpu(fts_ctx* c, size_t n, const fts_action_witness* w, uint64_t seed, uint8_t* out,
                                 size_t out_cap, size_t* offsets, size_t* lens) {
  if (c && !c->shards.empty()) c = c->shards[0];
  return actions_prove_device(c, n, w, 0, seed, out, out_cap, offsets, lens);
}
int fts_issue_prove_batch_gpu(fts_ctx* c, size_t n, const fts_action_witness* w, uint64_t seed, uint8_t* out,
                              size_t out_cap, size_t* offsets, size_t* lens) {
  if (c && !c->shards.empty()) c = c->shards[0];
  return actions_prove_device(c, n, w, 1, seed, out, out_cap, offsets, lens);
}
}  // extern "C"

extern "C" {
// token.Metadata.Deserialize + the opening check (auditor GetAuditInfoFor* + InspectOutput)
int fts_token_metadata_open_batch(fts_ctx* c, size_t n, const uint8_t* com64, const uint8_t* const* meta,
                                  const size_t* meta_len, int32_t* status) {
  if (!c || n > (size_t)(1u << 26) || (n && (!com64 || !meta || !meta_len || !status))) return FTS_API_EINVAL;
  if (n == 0) return FTS_API_OK;
  if (!c->shards.empty())
    return run_shards(plan(n, nullptr, (int)c->shards.size()), [&](int j, size_t lo, size_t hi) {
      return fts_token_metadata_open_batch(c->shards[j], hi - lo, com64 + 64 * lo, meta + lo, meta_len + lo, status + lo);
    });
  std::vector<req::TokenMeta> md(n);
  std::vector<fts_token_opening> items(n);
  parallel_for(n, 1024, [&](size_t i) {
    fts_token_opening& it = items[i];
    memset(&it, 0, sizeof it);
    req::TokenMeta& m = md[i];
    if (!meta[i] || !req::token_metadata(meta[i], meta_len[i], m)) return;  // NULL com64 -> FTS_E_MALFORMED
    it.com64 = com64 + 64 * i;
    it.type = m.type;
    it.type_len = m.type_len;
    it.value32 = m.has_value ? m.value : nullptr;
    it.bf32 = m.has_bf ? m.bf : nullptr;
  });
  return fts_token_open_batch(c, n, items.data(), status);
}

int fts_token_metadata_decode(const uint8_t* meta, size_t meta_len, int32_t* status, size_t* type_off,
                              size_t* type_len, uint8_t* value32, uint8_t* bf32, int32_t* has) {
  if (!status || !type_off || !type_len || !value32 || !bf32 || !has) return FTS_API_EINVAL;
  req::TokenMeta m;
  *status = meta && req::token_metadata(meta, meta_len, m) ? FTS_OK : FTS_E_MALFORMED;
  *type_off = m.type ? (size_t)(m.type - meta) : 0;
  *type_len = m.type_len;
  memcpy(value32, m.has_value ? m.value : req::kZero64, 32);
  memcpy(bf32, m.has_bf ? m.bf : req::kZero64, 32);
  *has = (m.has_value ? 1 : 0) | (m.has_bf ? 2 : 0);
  return FTS_API_OK;
}
}  // extern "C"
