// nlh_api.cpp -- C ABI of libnlh (include/nlh.h): device memory, streams,
// per-step orchestration, halo exchange over RCCL and error norms.
//
// One explicit-Euler step (reference do_work, src/2d_nonlocal_serial.cpp:
// 273-303; tile form src/2d_nonlocal_distributed.cpp:1146-1262):
//
//   single block (1 GPU): one stencil launch over the whole block.  The
//     out-of-domain halo is a static zero frame, so no exchange happens.
//
//   several blocks / ranks:
//     comm stream : pack halo pieces for other ranks -> grouped ncclSend /
//                   ncclRecv per peer -> unpack + local block-to-block copies
//     main stream : interior kernel (nodes whose disk lies inside the block,
//                   the reference's "interior" of :1156-1178) overlapped with
//                   the exchange, then the boundary bands (:1180-1259) once
//                   the halo event fires.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <execinfo.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <csignal>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nlh.h"
#include "nlh_device.h"
#include "nlh_plan.h"
#include "nlh_rt.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

int comm_init_bounded(ncclComm_t *out, int nranks, const ncclUniqueId &id, int rank, int device);

}  // namespace

namespace nlh {
// the 1D solver's entry points (nlh_1d.cpp) report through nlh_last_error too
const char *set_last_error(const std::string &msg) {
  g_err = msg;
  return g_err.c_str();
}
}  // namespace nlh

namespace {

#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess)                                                    \
      return fail(NLH_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define NCCL_TRY(expr)                                                       \
  do {                                                                       \
    ncclResult_t r_ = (expr);                                                \
    if (r_ != ncclSuccess)                                                   \
      return fail(NLH_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }
int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Stencil kernel, steps per pass and halo width for a parameter set: one
// resolution shared by nlh_create and the host-only plan queries, so the
// plans tests inspect are the ones production builds.
struct Resolved {
  int kernel = NLH_KERNEL_EXACT;
  bool pair = false;  // two steps per pass (nlh_pair.h)
  bool wide = false;  // large-horizon single-step kernel (nlh_wide.h)
  bool weighted = false;  // non-constant J: k_weighted (fast) instead of the J = 1 kernels
  bool prefix = false;  // run-time-horizon k_prefix_rt (eps past the k_wide instances)
  int halo = 0;       // eps, or 2*eps with pair
};

int resolve_config(const nlh_params &p, Resolved &r) {
  const int E = (int)p.eps;
  int kern = p.kernel;
  if (p.influence != NLH_INFLUENCE_CONSTANT && p.influence != NLH_INFLUENCE_LINEAR)
    return fail(NLH_ERR_ARG, "influence must be NLH_INFLUENCE_CONSTANT or NLH_INFLUENCE_LINEAR");
  if (p.influence != NLH_INFLUENCE_CONSTANT) {
    // a non-constant J has no nested-window form: k_weighted (fast) or
    // k_exact with the per-point J table
    if (kern == NLH_KERNEL_AUTO) kern = nlh::weighted_supported(E) ? NLH_KERNEL_FAST : NLH_KERNEL_EXACT;
    if (kern == NLH_KERNEL_FAST && !nlh::weighted_supported(E))
      return fail(NLH_ERR_UNSUPPORTED, "fast weighted kernel not instantiated for eps=" + std::to_string(E));
    r.kernel = kern;
    r.weighted = kern == NLH_KERNEL_FAST;
    r.halo = E;
    return NLH_OK;
  }
  // AUTO: the fast kernels in production AND test mode (the manufactured
  // source in its precomputed L_h[W0] form, within 1e-12 of field scale and
  // L2 within 1e-10 of the reference; EXACT remains selectable for bitwise
  // parity)
  if (kern == NLH_KERNEL_AUTO) kern = NLH_KERNEL_FAST;
  if (kern == NLH_KERNEL_FAST && !nlh::fast_supported(E) && !nlh::prefix_rt_supported(E)) {
    // beyond the nested-window horizons: the LDS-tile kernel with J = 1
    if (nlh::weighted_supported(E)) {
      r.kernel = kern;
      r.weighted = true;
      r.halo = E;
      return NLH_OK;
    }
    if (p.kernel == NLH_KERNEL_FAST)
      return fail(NLH_ERR_UNSUPPORTED, "fast kernel not instantiated for eps=" + std::to_string(E));
    kern = NLH_KERNEL_EXACT;
  }
  const double alpha = ((p.k * 8) / pow(p.eps * p.dh, 4)) * (p.dh * p.dh) * p.dt;
  const bool fold_ok = alpha != 0.0 && std::isfinite(1.0 / alpha);  // centre fold usable
  const bool folds = nlh::wide_supported(E) || nlh::prefix_rt_supported(E);
  if (kern == NLH_KERNEL_FAST && folds && !fold_ok) {
    // the large-horizon kernels fold the centre term (1/alpha - N)
    if (p.kernel == NLH_KERNEL_FAST)
      return fail(NLH_ERR_UNSUPPORTED, "fast kernel for eps > 16 needs k*dt*dh != 0");
    kern = NLH_KERNEL_EXACT;
  }
  r.kernel = kern;
  r.wide = kern == NLH_KERNEL_FAST && nlh::wide_supported(E);
  r.prefix = kern == NLH_KERNEL_FAST && nlh::prefix_rt_supported(E);
  // fast mode advances two steps per pass (test mode too: the manufactured
  // source of both steps folded into the pass); a zero alpha (no centre fold)
  // keeps the single-step kernels
  r.pair = kern == NLH_KERNEL_FAST && nlh::pair_supported(E) && fold_ok;
  if (const char *pe = std::getenv("NLH_PAIR")) r.pair = r.pair && std::atoi(pe) != 0;
  r.halo = r.pair ? 2 * E : E;
  return NLH_OK;
}

// Environment knobs libnlh reads (tuning and one-GPU verification).  Each one
// changes only the schedule -- strip width, ring depth, segment sizing,
// streams, the block decomposition over virtual ranks -- and the field stays
// within the FAST tolerance of the run without it (bitwise for the EXACT
// kernels): tests/test_gpu_parity.py::test_env_knobs_keep_results.  The
// round-2 ablation switches (NLH_ABLATE, NLH_PAIR_ABLATE), which made the
// library return meaningless fields, are gone; nlh_create refuses them, and
// any knob value outside its range, instead of ignoring them.
struct EnvKnob {
  const char *name;
  long lo, hi;
};
constexpr EnvKnob kEnvKnobs[] = {
    {"NLH_PAIR", 0, 1},            // 0: single-step kernels instead of the two-step pass
    {"NLH_FAST_R", 1, 4},          // k_fast columns per lane (1, 2 or 4)
    {"NLH_FORCE_BANDS", 0, 31},    // exchange-path schedule on a single block: 1 all sides, or 2 L | 4 R | 8 T | 16 B
    {"NLH_RCCL_SELF", 0, 1},       // one rank: halo pieces over RCCL to self
    {"NLH_VIRTUAL_RANKS", 0, 1024},  // run V virtual ranks in this process
    {"NLH_INT_PER_CU", 0, 64},     // interior workgroups per CU beside an exchange
    {"NLH_SCHED", 0, 2},           // where the edge bands run
    {"NLH_COMM_PRIO", 0, 1},       // exchange streams at the highest priority
    {"NLH_PAIR_SPLIT", 1, 4},      // 1: production pass with 16-slot rings (4: 8-slot, the default)
    {"NLH_PAIR_CU", 1, 16},        // pass workgroups per CU the segments are sized for
    {"NLH_PAIR_TEST", 0, 1},       // 0: test-mode pass with 16-slot rings
    {"NLH_PITCH_PAD", 0, 1024},    // extra doubles per padded row
    {"NLH_BAND_SEG", 0, 1 << 20},  // edge-band segment height (0 = automatic)
    {"NLH_COMM_INIT_TIMEOUT", 1, 86400},  // seconds a communicator init may take (default 300)
    {"NLH_SYNC", 0, 4},            // nlh_synchronize: 0 polls the streams (default), 1-4 set the device's
                                   // host-wait flag (yield, blocking, auto, spin) and block in HIP
    {"NLH_HOST_PROBE", 0, 1},      // diagnostics: nlh_run spins until its first launch has started
    {"NLH_GRAPH", 0, 1},           // 1: production passes replayed from captured HIP graphs
    {"NLH_SEGV_TRACE", 0, 1},      // diagnostics: a native backtrace on stderr on SIGSEGV / SIGBUS
    {"NLH_PAIR_PRIO", 0, 2},       // k_pair_split wave priority: 0 never, 1 one-round lists (default), 2 not on bands
    {"NLH_TRACE_REPART", 0, 1},    // repartition phase times on stderr
    {"NLH_PREFIX_WAVES", 0, 16},   // prefix kernels: waves per workgroup sharing a staged row (1, 2, 4, 8, 16; 0: by eps)
    {"NLH_PREFIX_ROWS", 0, 128},   // k_prefix_rt / k_prefix_rtc output rows per work item (32, 64; 96, 128 past
                                   // eps 224; 0: by eps)
};
constexpr const char *kRemovedKnobs[] = {"NLH_ABLATE", "NLH_PAIR_ABLATE"};

// NLH_SEGV_TRACE=1 (diagnostics): a native backtrace on stderr when the
// process takes SIGSEGV / SIGBUS, then the default action (a Python
// faulthandler shows only the interpreter's frames)
void segv_trace(int sig) {
  void *f[64];
  const int n = backtrace(f, 64);
  const char msg[] = "libnlh NLH_SEGV_TRACE: fatal signal, native backtrace:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(f, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void install_segv_trace() {
  static std::once_flag once;
  std::call_once(once, [] {
    signal(SIGSEGV, segv_trace);
    signal(SIGBUS, segv_trace);
  });
}

int check_env() {
  for (const char *name : kRemovedKnobs)
    if (std::getenv(name))
      return fail(NLH_ERR_ARG, std::string(name) +
                                   " is set: ablation diagnostics are not part of libnlh (tools/pair_bench.hip)");
  for (const EnvKnob &k : kEnvKnobs) {
    const char *v = std::getenv(k.name);
    if (!v || !*v) continue;
    char *end = nullptr;
    const long x = std::strtol(v, &end, 10);
    if (*end != '\0' || x < k.lo || x > k.hi)
      return fail(NLH_ERR_ARG, std::string(k.name) + "=" + v + ": expected an integer in [" + std::to_string(k.lo) +
                                   ", " + std::to_string(k.hi) + "]");
  }
  if (const char *v = std::getenv("NLH_PAIR_SPLIT"))
    if (*v && std::atoi(v) != 1 && std::atoi(v) != 4) return fail(NLH_ERR_ARG, "NLH_PAIR_SPLIT must be 1 or 4");
  return NLH_OK;
}

// NLH_VIRTUAL_RANKS=V (one process, one GPU): the owner map is resolved over
// V virtual ranks and this process runs all of them -- every virtual rank
// keeps its own blocks, per-peer message buffers, pack/unpack lists and busy
// time exactly as a real rank would (build_exchange with me = v); what a real
// run sends from rank A to rank B travels from A's send buffer into B's
// receive buffer through ncclSend/ncclRecv to self, grouped as a real run's
// exchange.  Gather, error norms, repartition and rebalance take the same
// per-rank paths.  RCCL refuses two ranks on one device, so this is how the
// multi-rank code runs on a one-GPU box.
int virtual_ranks(const nlh_params &p) {
  if (p.nranks != 1) return 0;
  const char *v = std::getenv("NLH_VIRTUAL_RANKS");
  const int n = v ? std::atoi(v) : 0;
  return n > 1 ? n : 0;
}

struct LocalBlock {
  int plan_index = 0;
  int owner = 0;  // (virtual) rank owning the block
  nlh::GRect r;
  int64_t pitch = 0, rows = 0;
  int32_t xl = 0;
  double *base[2] = {nullptr, nullptr};
  double *lw_base = nullptr;
  double *origin(int k) const { return base[k] + (int64_t)(rows - r.h) / 2 * pitch + xl; }
  double *lw_origin() const { return lw_base ? lw_base + (int64_t)(rows - r.h) / 2 * pitch + xl : nullptr; }
  // band flags: halo on that side depends on other blocks
  bool L = false, Rr = false, T = false, B = false;
};

// std::atomic<bool> that copies by value, so a rebuilt solver can be moved
// into the caller's handle (nlh_repartition)
struct Flag {
  std::atomic<bool> v{false};
  Flag() = default;
  Flag(const Flag &o) : v(o.v.load()) {}
  Flag &operator=(const Flag &o) {
    v = o.v.load();
    return *this;
  }
  Flag &operator=(bool b) {
    v = b;
    return *this;
  }
  operator bool() const { return v.load(); }
};

constexpr size_t kEvFold = 4096;  // timing events kept before folding (nlh_run)

// what one timing event pair brackets
enum EvKind : int8_t { kEvRun = 0, kEvInterior = 1, kEvBand = 2, kEvExchange = 3 };
struct EvMeta {
  int32_t owner = -1;     // busy timing: the (virtual) rank of the launches
  int16_t launches = 0;   // busy timing: kernel launches inside the pair
  int8_t kind = kEvRun;
  bool open = false;      // second event not recorded yet
};

struct Peer {
  int me = 0;     // the (virtual) rank of this process holding the buffers
  int rank = 0;   // the peer rank
  int mate = -1;  // virtual ranks: index of the (rank, me) entry receiving what me sends
  int64_t send_count = 0, recv_count = 0;  // doubles
  double *send = nullptr, *recv = nullptr;
};

}  // namespace

struct nlh_solver {
  nlh_params p{};
  std::vector<int32_t> owner;
  nlh::Plan plan;
  std::vector<LocalBlock> blocks;
  int device = 0;
  int cus = 256;  // compute units of the device
  int kernel = NLH_KERNEL_EXACT;
  int fast_r = 2;  // columns per lane of the fast kernel (NLH_FAST_R=1|2|4: 64/128/256-column strips)
  bool pair = false;  // two steps per pass (nlh_pair.h); production fast mode (NLH_PAIR=0 disables)
  bool wide = false;  // k_wide (nlh_wide.h) for eps 17..48
  bool weighted = false;  // k_weighted: non-constant influence function
  bool prefix = false;    // k_prefix_rt (nlh_prefix.h) past the k_wide horizons
  int32_t *d_ptab = nullptr;  // k_prefix_rt's per-offset prefix index table
  int prefix_rows = 0;        // its R (output rows per work item: nlh::prefix_rt_rows)
  int prefix_waves = 1;       // waves per workgroup sharing a staged row (nlh::prefix_rt_waves)
  double *d_lsx = nullptr, *d_lty = nullptr;  // fast test mode, J = 1: separable L_h[W0] tables (sep_tables)
  int sep_nlv = 0, sep_lts = 0;                // their level count and lty row stride
  double *d_wt = nullptr, *d_qj = nullptr;  // J tables (influence != 0)
  int halo = 0;       // halo rows/columns held per block: eps, or 2*eps with pair
  // production k_pair_split rings: 6 = D4/B2 (default; with row pairs 444-450 vs 438-446 G
  // node/s for D8/B4 at C2, profiles/r03/rowpairs/pair_rows_sweep.jsonl), 1 = D8/B4 (NLH_PAIR_SPLIT=1)
  int pair_split = 6;
  // test-mode pass: 5 = k_pair_split<TEST> with 8-slot rings (D=4, B=2; 322 vs
  // 287 G node/s at C2 for the production rings, profiles/r02/tune_test.jsonl),
  // 4 = D=8, B=4 (NLH_PAIR_TEST=0)
  int pair_test = 5;
  int pair_cu = 4;     // split-kernel workgroups per CU the segments are sized for (NLH_PAIR_CU)
  int64_t pair_resident = 0;  // k_pair_split workgroups the device holds at once (0: not yet asked)
  int pair_prio = 1;          // NLH_PAIR_PRIO (kEnvKnobs)
  hipStream_t s_main = nullptr, s_comm = nullptr, s_band = nullptr;
  hipEvent_t ev_ready = nullptr, ev_halo = nullptr, ev_band = nullptr, ev_int = nullptr;
  bool halo_fresh = false;  // the current field's halo holds its neighbours' values
  // diagnostics (NLH_FORCE_BANDS): exchange-path schedule on one block, bands
  // on the sides of the mask (1: all four; else 2 left, 4 right, 8 top, 16 bottom)
  int force_bands = 0;
  bool rccl_self = false;    // diagnostics (NLH_RCCL_SELF): one rank, local pieces over RCCL to self
  bool exchange_planned = false;  // the plan has halo pieces (set before the rect lists)
  int vranks = 0;       // NLH_VIRTUAL_RANKS count (0: one real rank per process)
  std::vector<int> mine;  // ranks this process runs: {rank}, or 0 .. vranks-1
  int owners = 1;  // owner ids in the tile map: nranks, or NLH_VIRTUAL_RANKS
  // exchange schedule: interior workgroups per CU in the segment model when
  // an exchange runs beside it (NLH_INT_PER_CU, 0 = all the pass kernel's
  // slots), and where the bands run (NLH_SCHED): 0 = own stream beside the
  // interior (default since round 6), 2 = on the exchange stream (rounds
  // 1-5), 1 = before the interior on s_main.  Round 6, one rank's pass with
  // the exchange-path schedule forced on its sides (tools/rank_proxy.py,
  // profiles/r06/rank_proxy/sched/): a C3 rank (16384 x 8192, 2-3 sides)
  // 502-505 us per pass with 0 against 600-611 with 2 (518 alone), a 9216^2
  // C5 tile with 3 sides 357-360 against 405-413, 4096^2 ranks with 1-3 sides
  // 78.5-79.3 against 79.8-81.1; only a four-sided 4096^2 block ran worse
  // (84.9 / 91.6 against 80.8-82.6), a layout the 2x1 / 2x2 / 2x4 runs do not
  // have; the virtual-rank lines (C3, C5, weak 2 / 4 / 8) within +-1% except
  // C3's, +3.4%.  Round 4: all slots (0) beat round 1's 3 per CU on one rank's
  // blocks over RCCL to self -- 4096^2 as 2x1 blocks 82 vs 88-90 us per pass,
  // 8192x4096 as 2x1 156-157 vs 164-166, 8192^2 as 2x2 290-295 vs 296-298
  // (profiles/r04/sched); the pass kernel's 4 workgroups per CU hold 252 of
  // 512 VGPRs per SIMD lane and 56 of 160 KB of LDS, so bands and RCCL
  // kernels still find room beside them
  int int_per_cu = 0;
  int sched = 0;
  int64_t t = 0;
  int cur = 0;
  double *d_sxt = nullptr, *d_syt = nullptr;
  int32_t *d_lens = nullptr;
  nlh::StepConst sc{};
  int64_t disk = 0;
  bool exchange = false;
  // launches per phase and parity (chunked at kMaxRects / kMaxCopies)
  std::vector<nlh::RectList> rl_full[2], rl_int[2], rl_bnd[2];
  std::vector<nlh::RectList> pl_full[2], pl_int[2], pl_bnd[2];  // pair-kernel launches
  // halo exchange
  ncclComm_t comm = nullptr;
  std::vector<Peer> peers;
  std::vector<nlh::CopyList> cl_pack[2], cl_unpack[2], cl_local[2];
  int64_t halo_bytes = 0;
  // norms
  nlh::NormPartial *d_part = nullptr;
  std::vector<int> part_off;
  int part_total = 0;
  double *d_red = nullptr;
  // timing: 0 off, 1 one event pair per nlh_run, 2 busy (serialised passes, a
  // pair per (virtual) rank's launch group), 3 phases (a pair per pass's
  // interior, bands and exchange, one per nlh_run)
  int timing = 0;
  std::vector<hipEvent_t> ev_pool;  // pair p = events 2p, 2p + 1
  double *stage = nullptr;  // repartition staging buffer, kept for the next one (kStageKeepBytes)
  size_t stage_cap = 0;     // its size in doubles
  size_t ev_used = 0;
  std::vector<EvMeta> ev_meta;      // one per recorded pair
  // pairs already folded into running totals (long windows: completed pairs
  // are folded every kEvFold events instead of the pool growing with the run)
  double ev_acc_kind[4] = {0.0, 0.0, 0.0, 0.0};  // per EvKind
  std::vector<double> ev_acc_owner;  // folded busy milliseconds per owner
  int64_t timed_steps = 0, timed_passes = 0;  // since timing was enabled
  double launch_overhead_ms = 0.0;  // busy timing: the cost of one more (empty) launch in a pair
  double pair_overhead_ms = 0.0;    // busy timing: an event pair's own cost (once per pair)
  int32_t comm_nranks = 0, comm_rank = -1;  // as RCCL reports them
  int64_t device_bytes = 0;
  char arch[32] = {0};
  // logging snapshots (nlh_snapshot_begin / _wait): owned nodes packed block
  // after block, device copy then pinned host copy on s_copy
  hipStream_t s_copy = nullptr;
  hipEvent_t ev_snap_dev = nullptr, ev_snap = nullptr;
  double *snap_dev = nullptr, *snap_host = nullptr;
  Flag snap_pending;
  // host waits and host-side timing (nlh_host_time): steady-clock ns of the
  // last nlh_run's entry / return, of nlh_synchronize's first observation of
  // that run's end event (timing 1) and of its return
  int sync_mode = 0;        // NLH_SYNC (kEnvKnobs)
  bool host_probe = false;  // NLH_HOST_PROBE: record when the run's start event completes
  int64_t h_enter = 0, h_return = 0, h_start_seen = -1, h_end_seen = -1, h_sync_return = 0;
  hipEvent_t h_e0 = nullptr, h_e1 = nullptr;  // the last nlh_run's event pair (timing 1 / 3)
  // HIP graphs of production passes (NLH_GRAPH=1, single-stream solvers):
  // runs of g passes (g a power of two, 2 .. kGraphMaxPasses) starting at
  // buffer parity k, captured on first use and replayed by one hipGraphLaunch
  // each (capture_graph)
  struct Graph {
    int passes = 0, k = 0;
    hipGraphExec_t exec = nullptr;
  };
  bool graph_on = false;
  std::vector<Graph> graphs;
};

namespace {

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int set_device(const nlh_solver *s) {
  HIP_TRY(hipSetDevice(s->device));
  return NLH_OK;
}

void fill_rect_common(nlh::Rect &R, const LocalBlock &b, int k, const nlh_solver *s) {
  R.u = b.origin(k);
  R.un = b.origin(1 - k);
  R.lw = b.lw_origin();
  R.pitch = b.pitch;
  R.gx0 = (int32_t)b.r.x0;
  R.gy0 = (int32_t)b.r.y0;
  (void)s;
}

// split one block into interior + bands (interior first)
struct LRect { int x0, y0, x1, y1; bool interior; };

std::vector<LRect> split_block(const LocalBlock &b, int E, int sw) {
  const int bx = (int)b.r.w, by = (int)b.r.h;
  std::vector<LRect> out;
  if (!(b.L || b.Rr || b.T || b.B)) {
    out.push_back({0, 0, bx, by, true});
    return out;
  }
  int a = b.L ? std::min(sw, bx) : 0;
  if (b.L && a < E) a = std::min(E, bx);
  int bb = bx;
  if (b.Rr) {
    const int lim = bx - E;
    bb = lim <= a ? a : a + (lim - a) / sw * sw;
  }
  int yt = b.T ? std::min(E, by) : 0;
  int yb = b.B ? std::max(by - E, yt) : by;
  if (bb > a && yb > yt) out.push_back({a, yt, bb, yb, true});
  if (a > 0) out.push_back({0, 0, a, by, false});
  if (bb < bx) out.push_back({bb, 0, bx, by, false});
  if (bb > a && yt > 0) out.push_back({a, 0, bb, yt, false});
  if (bb > a && yb < by) out.push_back({a, yb, bb, by, false});
  return out;
}

// kind 0: single-step kernels (k_exact / k_fast); kind 1: the pair kernel
int build_rectlists(nlh_solver *s, int kind) {
  const int E = (int)s->p.eps;
  // k_weighted tiles like k_exact (64-column strips, fixed segments)
  const bool fast = s->kernel == NLH_KERNEL_FAST && !s->weighted;
  const bool pair = kind == 1;
  const int sw = pair        ? nlh::pair_strip_width(E)
                 : !fast     ? 64
                 : s->prefix ? nlh::prefix_rt_strip_width(E, s->prefix_waves)
                             : nlh::fast_strip_width(E, s->fast_r);
  // gather local rects (bands are s->halo wide: what the halo exchange refreshes)
  struct Item { int blk; LRect r; };
  std::vector<Item> all, inter, bnd;
  for (size_t bi = 0; bi < s->blocks.size(); ++bi) {
    for (auto &r : split_block(s->blocks[bi], s->halo, sw)) {
      Item it{(int)bi, r};
      all.push_back(it);
      (r.interior ? inter : bnd).push_back(it);
    }
  }
  // Segment heights (interior, bands) for a set of rects sized as ONE rank's
  // launch on the whole GPU.  Virtual ranks are sized each for itself, as
  // each would be on its own GPU: then each one's launches fill the device and
  // its measured busy time follows its own work (load balancing).
  auto sizes = [&](const std::vector<Item> &all, const std::vector<Item> &inter,
                   const std::vector<Item> &bnd) -> std::pair<int, int> {
    // segment height for the fast kernel: ~1024 single-wave workgroups (4 per CU,
    // all resident at once; balanced grids measured fastest, profiles/r01/tune_*.json)
    int seg_h = 4;
    if (fast) {
      int64_t strip_rows = 0;
      for (auto &it : all) strip_rows += ceil_div(it.r.x1 - it.r.x0, sw) * (it.r.y1 - it.r.y0);
      const bool own = s->p.seg_rows > 0 && pair == s->pair;  // seg_rows tunes the kernel nlh_run uses most
      if (pair) {
        // k_pair_split: 4 workgroups (8 waves) per CU -- taller segments beat
        // more waves (profiles/r01/tune_v3b).  Segment height: minimise rounds
        // x sweep, a sweep costing seg + 3E rows (stage 1 reads seg + 4E rows,
        // stage 2 seg + 2E); at 4096^2 this picks 152 rows = 999 workgroups in
        // one round, the measured optimum; on large lattices several rounds of
        // shorter segments instead of one round with idle slots
        const int per_cu = std::max(1, nlh::pair_blocks_per_cu(E, s->p.test ? s->pair_test : s->pair_split));
        int use_cu = std::min(per_cu, s->pair_cu);
        // with an exchange the interior may be sized for fewer slots per CU,
        // leaving room for the bands and RCCL beside it (NLH_INT_PER_CU; off by
        // default since round 4, see int_per_cu) -- never on blocks past
        // 4096 x 8192 (a loss on the 16384 x 8192 share of C3)
        int64_t big = 0;
        for (auto &it : all) big = std::max<int64_t>(big, s->blocks[it.blk].r.w * s->blocks[it.blk].r.h);
        if (s->exchange_planned && s->int_per_cu > 0 && big <= (int64_t)4096 * 8192)
          use_cu = std::min(use_cu, s->int_per_cu);
        const int64_t resident = (int64_t)use_cu * s->cus;
        const std::vector<Item> &sized = inter.empty() ? all : inter;
        int64_t hmax = 1;
        for (auto &it : sized) hmax = std::max<int64_t>(hmax, it.r.y1 - it.r.y0);
        int64_t best = -1, best_cost = 0;
        for (int64_t n = 1; n <= 1024; ++n) {
          const int64_t seg = std::max<int64_t>(16, ceil_div(hmax, n));
          int64_t wgs = 0;
          for (auto &it : sized) wgs += ceil_div(it.r.x1 - it.r.x0, sw) * ceil_div(it.r.y1 - it.r.y0, seg);
          const int64_t cost = ceil_div(wgs, resident) * (seg + 3 * E);
          if (best < 0 || cost < best_cost) {
            best = seg;
            best_cost = cost;
          }
          if (seg == 16) break;
        }
        seg_h = own ? s->p.seg_rows : (int)best;
      } else if (s->prefix) {
        seg_h = s->prefix_rows;  // the kernel's register block of output rows
      } else if (s->wide) {
        // k_wide: one-wave workgroups, all resident in one round: two waves per
        // SIMD up to E = 40 (8 per CU, 214 VGPRs at E = 32;
        // profiles/r02/wide_bench_*), one beyond (4 per CU)
        const int per_cu = std::max(1, std::min(8, nlh::wide_blocks_per_cu(E)));
        seg_h = own ? s->p.seg_rows
                    : (int)std::max<int64_t>(2 * E, ceil_div(strip_rows, (int64_t)per_cu * s->cus));
      } else {
        seg_h = own ? s->p.seg_rows
                    : (int)std::max<int64_t>(nlh::fast_seg_min(E), ceil_div(strip_rows, 1024));
      }
    }
    // halo bands run beside the interior kernel (enqueue_step); their segments
    // are short -- about one band workgroup per CU -- so that bands, the
    // exchange they feed and the next pass's bands fit inside one interior
    // pass, but (two-step pass) not below 4E rows: a three-sided 4096^2 rank (left strip +
    // top / bottom bands: 21-row segments) ran 89-97 us per pass against
    // 80-83 with 32-64-row band segments, one side or four 78-85 either way
    // (round 6, profiles/r06/rank_proxy/seg/).  NLH_BAND_SEG overrides the
    // height (diagnostics)
    int seg_band = seg_h;
    if (fast) {
      int64_t band_rows = 0;
      for (auto &it : bnd) band_rows += ceil_div(it.r.x1 - it.r.x0, sw) * (it.r.y1 - it.r.y0);
      const int lo = std::min(seg_h, (pair ? 4 : 2) * E);
      seg_band = (int)std::min<int64_t>(seg_h, std::max<int64_t>(lo, ceil_div(band_rows, (int64_t)s->cus)));
      if (const char *bsg = std::getenv("NLH_BAND_SEG"))
        if (std::atoi(bsg) > 0) seg_band = std::atoi(bsg);
      if (s->prefix) seg_band = seg_h;  // fixed R-row blocks
    }
    return {seg_h, seg_band};
  };
  std::map<int, std::pair<int, int>> seg_of;  // (virtual) rank -> (interior, band) heights
  if (s->vranks) {
    for (int v : s->mine) {
      std::vector<Item> a, in, bd;
      for (auto &it : all) {
        if (s->blocks[it.blk].owner != v) continue;
        a.push_back(it);
        (it.r.interior ? in : bd).push_back(it);
      }
      if (!a.empty()) seg_of[v] = sizes(a, in, bd);
    }
  }
  const std::pair<int, int> seg_all = sizes(all, inter, bnd);
  (pair ? s->sc.seg_pair : s->sc.seg_h) = seg_all.first;
  auto make = [&](const std::vector<Item> &items, int k, std::vector<nlh::RectList> &out) -> int {
    out.clear();
    int w = 0;
    for (auto &it : items) {
      // a list never mixes (virtual) ranks: busy time is measured per rank
      const int own = s->blocks[it.blk].owner;
      if (out.empty() || out.back().nrects >= nlh::kMaxRects || out.back().owner != own) {
        if (!out.empty()) out.back().nwork = w;
        out.emplace_back();
        std::memset(&out.back(), 0, sizeof(nlh::RectList));
        out.back().owner = own;
        w = 0;
      }
      nlh::RectList &rl = out.back();
      nlh::Rect &R = rl.r[rl.nrects++];
      fill_rect_common(R, s->blocks[it.blk], k, s);
      R.x0 = it.r.x0; R.y0 = it.r.y0; R.x1 = it.r.x1; R.y1 = it.r.y1;
      if (fast) {
        const std::pair<int, int> &sg = s->vranks ? seg_of[own] : seg_all;
        R.seg_rows = it.r.interior ? sg.first : sg.second;
        R.nstrip = (int)ceil_div(R.x1 - R.x0, sw);
        R.nseg = (int)ceil_div(R.y1 - R.y0, R.seg_rows);
      } else {
        R.seg_rows = (s->weighted || nlh::exact_lds_ok(E, s->p.test != 0)) ? 16 : 4;
        R.nstrip = (int)ceil_div(R.x1 - R.x0, 64);
        R.nseg = (int)ceil_div(R.y1 - R.y0, R.seg_rows);
      }
      R.wg_begin = w;
      w += R.nstrip * R.nseg;
    }
    if (!out.empty()) out.back().nwork = w;
    return NLH_OK;
  };
  for (int k = 0; k < 2; ++k) {
    int rc;
    if ((rc = make(all, k, pair ? s->pl_full[k] : s->rl_full[k])) != NLH_OK) return rc;
    if ((rc = make(inter, k, pair ? s->pl_int[k] : s->rl_int[k])) != NLH_OK) return rc;
    if ((rc = make(bnd, k, pair ? s->pl_bnd[k] : s->rl_bnd[k])) != NLH_OK) return rc;
  }
  return NLH_OK;
}

int add_copy(std::vector<nlh::CopyList> &v, const double *src, int64_t spitch, double *dst,
             int64_t dpitch, int64_t w, int64_t h) {
  if (w <= 0 || h <= 0) return NLH_OK;
  if (v.empty() || v.back().ncopies >= nlh::kMaxCopies) {
    v.emplace_back();
    std::memset(&v.back(), 0, sizeof(nlh::CopyList));
  }
  nlh::CopyList &cl = v.back();
  nlh::Copy &c = cl.c[cl.ncopies++];
  c.src = src;
  c.dst = dst;
  c.spitch = spitch;
  c.dpitch = dpitch;
  c.w = (int32_t)w;
  c.h = (int32_t)h;
  c.wg_begin = cl.nwork;
  cl.nwork += (int32_t)ceil_div(w * h, 256);
  return NLH_OK;
}

// pointer to global node (gx, gy) inside local block b, parity k
double *node_ptr(const LocalBlock &b, int k, int64_t gx, int64_t gy) {
  return b.origin(k) + (gy - b.r.y0) * b.pitch + (gx - b.r.x0);
}

int build_exchange(nlh_solver *s) {
  std::map<int, size_t> local_of_plan;  // plan block index -> local index
  for (size_t i = 0; i < s->blocks.size(); ++i) local_of_plan[s->blocks[i].plan_index] = i;
  // a piece travels over RCCL when its blocks sit on different (virtual)
  // ranks; with NLH_RCCL_SELF (one real rank) every piece goes through
  // ncclSend/ncclRecv to self instead of a local copy
  const bool self_all = s->rccl_self && s->vranks == 0;
  std::vector<std::vector<nlh::XferEntry>> lay(s->mine.size());
  std::map<std::pair<int, int>, Peer> peers;  // (me, peer rank)
  for (size_t m = 0; m < s->mine.size(); ++m) {
    const int me = s->mine[m];
    lay[m] = nlh::exchange_layout(s->plan, me, self_all);
    for (const auto &e : lay[m]) {
      const nlh::Piece &pc = s->plan.pieces[e.piece];
      Peer &pr = peers[{me, e.peer}];
      pr.me = me;
      pr.rank = e.peer;
      int64_t &cnt = e.dir == 0 ? pr.send_count : pr.recv_count;
      cnt = std::max(cnt, e.offset + pc.r.w * pc.r.h);
    }
  }
  for (auto &kv : peers) {
    Peer &pr = kv.second;
    if (pr.send_count) HIP_TRY(hipMalloc(&pr.send, pr.send_count * sizeof(double)));
    if (pr.recv_count) HIP_TRY(hipMalloc(&pr.recv, pr.recv_count * sizeof(double)));
    s->device_bytes += (pr.send_count + pr.recv_count) * (int64_t)sizeof(double);
    s->halo_bytes += pr.send_count * (int64_t)sizeof(double);
    s->peers.push_back(pr);  // ordered by (me, peer)
  }
  if (s->vranks) {
    // what virtual rank A sends to B lands in B's receive buffer from A: the
    // two message layouts must agree (they do by construction: both walk the
    // plan in order -- checked here before any transfer is enqueued)
    for (size_t i = 0; i < s->peers.size(); ++i) {
      Peer &pr = s->peers[i];
      for (size_t j = 0; j < s->peers.size(); ++j)
        if (s->peers[j].me == pr.rank && s->peers[j].rank == pr.me) pr.mate = (int)j;
      const int64_t want = pr.mate >= 0 ? s->peers[pr.mate].recv_count : 0;
      if (pr.send_count != want)
        return fail(NLH_ERR_STATE, "internal: virtual rank " + std::to_string(pr.me) + " sends " +
                                       std::to_string(pr.send_count) + " doubles to " + std::to_string(pr.rank) +
                                       ", which expects " + std::to_string(want));
    }
  }
  auto peer_of = [&](int me, int rank) -> Peer & {
    for (auto &pr : s->peers)
      if (pr.me == me && pr.rank == rank) return pr;
    return s->peers.front();  // unreachable: every layout entry made a peer
  };
  for (int k = 0; k < 2; ++k) {
    auto &pk = s->cl_pack[k], &up = s->cl_unpack[k], &lc = s->cl_local[k];
    pk.clear();
    up.clear();
    lc.clear();
    for (size_t m = 0; m < s->mine.size(); ++m) {
      for (const auto &e : lay[m]) {
        const nlh::Piece &pc = s->plan.pieces[e.piece];
        Peer &pr = peer_of(s->mine[m], e.peer);
        int rc;
        if (e.dir == 0) {
          const LocalBlock &sb = s->blocks[local_of_plan[pc.src_block]];
          rc = add_copy(pk, node_ptr(sb, k, pc.r.x0, pc.r.y0), sb.pitch, pr.send + e.offset, pc.r.w, pc.r.w,
                        pc.r.h);
        } else {
          const LocalBlock &db = s->blocks[local_of_plan[pc.dst_block]];
          rc = add_copy(up, pr.recv + e.offset, pc.r.w, node_ptr(db, k, pc.r.x0, pc.r.y0), db.pitch, pc.r.w,
                        pc.r.h);
        }
        if (rc != NLH_OK) return rc;
      }
    }
    // pieces between blocks of one (virtual) rank: device copies
    for (const auto &pc : s->plan.pieces) {
      if (pc.src_rank != pc.dst_rank || self_all) continue;
      if (!local_of_plan.count(pc.src_block)) continue;  // another process's blocks
      const LocalBlock &sb = s->blocks[local_of_plan[pc.src_block]];
      const LocalBlock &db = s->blocks[local_of_plan[pc.dst_block]];
      const int rc = add_copy(lc, node_ptr(sb, k, pc.r.x0, pc.r.y0), sb.pitch, node_ptr(db, k, pc.r.x0, pc.r.y0),
                              db.pitch, pc.r.w, pc.r.h);
      if (rc != NLH_OK) return rc;
    }
  }
  s->exchange = !s->plan.pieces.empty() || s->force_bands != 0;
  return NLH_OK;
}

hipEvent_t pool_event(nlh_solver *s) {
  if (s->ev_used == s->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    s->ev_pool.push_back(e);
  }
  return s->ev_pool[s->ev_used++];
}

// a timed event pair: begin() records its first event on `st` and its
// bookkeeping (open until end() records the second event; a fold inside
// nlh_run keeps open pairs -- the per-run pair -- in flight)
struct TimedPair {
  nlh_solver *s;
  hipEvent_t e1 = nullptr;
  int begin(hipStream_t st, EvKind kind, int owner = -1, int launches = 0) {
    hipEvent_t e0 = pool_event(s);
    e1 = pool_event(s);
    if (!e0 || !e1) return fail(NLH_ERR_HIP, "event pool");
    HIP_TRY(hipEventRecord(e0, st));
    EvMeta m;
    m.kind = kind;
    m.owner = owner;
    m.launches = (int16_t)std::min(launches, 32767);
    m.open = true;
    s->ev_meta.push_back(m);
    return NLH_OK;
  }
  int end(hipStream_t st) {
    HIP_TRY(hipEventRecord(e1, st));
    for (size_t p = s->ev_meta.size(); p-- > 0;)  // folds may have moved the pair
      if (s->ev_pool[2 * p + 1] == e1) {
        s->ev_meta[p].open = false;
        return NLH_OK;
      }
    return fail(NLH_ERR_STATE, "internal: timing pair lost");
  }
};

using RLIter = std::vector<nlh::RectList>::const_iterator;

int launch_stencil(nlh_solver *s, RLIter b, RLIter e, hipStream_t st) {
  const bool test = s->p.test != 0;
  for (; b != e; ++b) {
    const nlh::RectList &rl = *b;
    if (rl.nwork == 0) continue;
    int rc;
    if (s->weighted)
      rc = nlh::launch_weighted(rl, s->sc, test, st);
    else if (s->prefix)
      rc = nlh::launch_prefix_rt(rl, s->sc, s->d_ptab, test, s->prefix_waves, st);
    else if (s->wide)
      rc = nlh::launch_wide(rl, s->sc, test, st);
    else if (s->kernel == NLH_KERNEL_FAST)
      rc = nlh::launch_fast(rl, s->sc, test, s->fast_r, st);
    else
      rc = nlh::launch_exact(rl, s->sc, test, st);
    if (rc != 0) return fail(NLH_ERR_HIP, std::string("stencil launch failed: ") + hipGetErrorString((hipError_t)rc));
  }
  return NLH_OK;
}

int launch_pair_lists(nlh_solver *s, RLIter b, RLIter e, hipStream_t st, bool band) {
  for (; b != e; ++b) {
    const nlh::RectList &rl = *b;
    if (rl.nwork == 0) continue;
    // the wave priority of k_pair_split pays only when every workgroup of the
    // launch is resident at once (nlh_pair.h kPairNoPrio)
    int v = s->p.test ? s->pair_test : s->pair_split;
    if (v == 5 || v == 6) {
      if (s->pair_resident == 0)
        s->pair_resident = (int64_t)std::max(1, nlh::pair_blocks_per_cu((int)s->p.eps, v)) * s->cus;
      if (rl.nwork > s->pair_resident || s->pair_prio == 0 || (band && s->pair_prio == 2)) v |= nlh::kPairNoPrio;
    }
    const int rc = nlh::launch_pair(rl, s->sc, v, st);
    if (rc != 0) return fail(NLH_ERR_HIP, std::string("pair launch failed: ") + hipGetErrorString((hipError_t)rc));
  }
  return NLH_OK;
}

int launch_copy_lists(const std::vector<nlh::CopyList> &v, hipStream_t st) {
  for (const auto &cl : v)
    if (nlh::launch_copies(cl, st)) return fail(NLH_ERR_HIP, "halo copy launch");
  return NLH_OK;
}

void set_time(nlh_solver *s, int64_t t) {
  // (2*M_PI)*(time*dt) exactly as the reference spells it (:208, :237)
  const double arg = 2 * M_PI * (t * s->p.dt);
  s->sc.st2pi = 2 * M_PI * sin(arg);
  s->sc.ct = cos(arg);
  const double arg2 = 2 * M_PI * ((t + 1) * s->p.dt);
  s->sc.st2pi2 = 2 * M_PI * sin(arg2);
  s->sc.ct2 = cos(arg2);
}

// halo exchange of the field in buffer parity k on the comm stream: pack the
// pieces other ranks need -> grouped ncclSend / ncclRecv per peer -> unpack
// + local block-to-block copies; records ev_halo
int enqueue_exchange(nlh_solver *s, int k) {
  if (launch_copy_lists(s->cl_pack[k], s->s_comm)) return NLH_ERR_HIP;
  if (!s->peers.empty()) {
    NCCL_TRY(ncclGroupStart());
    if (s->vranks) {
      // every virtual A -> B message: A's send buffer for B into B's receive
      // buffer from A, through RCCL to self (send/recv pairs match in issue
      // order within the group)
      for (auto &pr : s->peers) {
        if (!pr.send_count) continue;
        NCCL_TRY(ncclSend(pr.send, pr.send_count, ncclDouble, 0, s->comm, s->s_comm));
        NCCL_TRY(ncclRecv(s->peers[pr.mate].recv, pr.send_count, ncclDouble, 0, s->comm, s->s_comm));
      }
    } else {
      for (auto &pr : s->peers) {
        if (pr.send_count) NCCL_TRY(ncclSend(pr.send, pr.send_count, ncclDouble, pr.rank, s->comm, s->s_comm));
        if (pr.recv_count) NCCL_TRY(ncclRecv(pr.recv, pr.recv_count, ncclDouble, pr.rank, s->comm, s->s_comm));
      }
    }
    NCCL_TRY(ncclGroupEnd());
  }
  if (launch_copy_lists(s->cl_unpack[k], s->s_comm)) return NLH_ERR_HIP;
  if (launch_copy_lists(s->cl_local[k], s->s_comm)) return NLH_ERR_HIP;
  HIP_TRY(hipEventRecord(s->ev_halo, s->s_comm));
  return NLH_OK;
}

// a pass's exchange; with phase timing (3) bracketed by its own event pair
int enqueue_exchange_timed(nlh_solver *s, int k) {
  if (s->timing != 3) return enqueue_exchange(s, k);
  TimedPair tp{s};
  int rc;
  if ((rc = tp.begin(s->s_comm, kEvExchange)) || (rc = enqueue_exchange(s, k))) return rc;
  return tp.end(s->s_comm);
}

// one time step (nsteps == 1, k_exact / k_fast) or two (nsteps == 2, the pair
// kernel).  With an exchange (several blocks / ranks), pass n runs
//   s_band : wait halo(n) and interior(n-1); bands(n)    (nodes within the
//            halo width of a block edge: they read the halo)
//   s_main : wait bands(n-1); interior(n)                (concurrently)
//   s_comm : wait bands(n); exchange -> halo(n+1)        (overlaps interior(n))
// so the exchange of the next pass's halo overlaps this pass's interior, and
// the bands -- short segments, see build_rectlists -- run beside it.  The
// pieces sent are band nodes only (every node within the halo width of a
// block side that is not on the domain boundary belongs to a band).
int enqueue_step(nlh_solver *s, int nsteps) {
  const int k = s->cur;
  const bool two = nsteps == 2;
  set_time(s, s->t);
  if (s->timing) {
    s->timed_steps += nsteps;
    ++s->timed_passes;
  }
  // one group of stencil launches (interior, bands or the full block) on st
  auto stencil = [&](const std::vector<nlh::RectList> &one, const std::vector<nlh::RectList> &pr,
                     hipStream_t st, EvKind kind) {
    const std::vector<nlh::RectList> &v = two ? pr : one;
    auto run = [&](RLIter b, RLIter e) {
      return two ? launch_pair_lists(s, b, e, st, kind == kEvBand) : launch_stencil(s, b, e, st);
    };
    bool any = false;
    for (const auto &rl : v) any |= rl.nwork > 0;
    if (s->timing == 3 && any) {  // phase timing: one pair around the group
      TimedPair tp{s};
      int r;
      if ((r = tp.begin(st, kind)) || (r = run(v.begin(), v.end()))) return r;
      return tp.end(st);
    }
    if (s->timing != 2) return run(v.begin(), v.end());
    // busy time: an event pair around each (virtual) rank's launches of this
    // group (its lists are contiguous, build_rectlists)
    for (RLIter b = v.begin(); b != v.end();) {
      RLIter e = b;
      int launches = 0;
      while (e != v.end() && e->owner == b->owner) launches += (e++)->nwork > 0;
      if (launches) {
        TimedPair tp{s};
        int r;
        if ((r = tp.begin(st, kind, b->owner, launches)) || (r = run(b, e)) || (r = tp.end(st))) return r;
      }
      b = e;
    }
    return (int)NLH_OK;
  };
  int rc;
  if (!s->exchange) {
    if ((rc = stencil(s->rl_full[k], s->pl_full[k], s->s_main, kEvInterior))) return rc;
  } else {
    if (!s->halo_fresh) {  // first pass after test_init / set_field: this input's halo
      HIP_TRY(hipEventRecord(s->ev_ready, s->s_main));
      HIP_TRY(hipStreamWaitEvent(s->s_comm, s->ev_ready, 0));
      if ((rc = enqueue_exchange(s, k))) return rc;
      s->halo_fresh = true;
    }
    if (s->timing == 2) {
      // busy timing: the pass serialised on s_main -- halo(n), every rank's
      // bands, every rank's interior -- so each rank's pairs time its own
      // kernels alone (not the other ranks' kernels running beside them on a
      // second stream) and no halo wait; the exchange of pass n + 1 runs on
      // s_comm beside the interiors
      HIP_TRY(hipStreamWaitEvent(s->s_main, s->ev_halo, 0));  // halo(n)
      if ((rc = stencil(s->rl_bnd[k], s->pl_bnd[k], s->s_main, kEvBand))) return rc;
      HIP_TRY(hipEventRecord(s->ev_band, s->s_main));
      if ((rc = stencil(s->rl_int[k], s->pl_int[k], s->s_main, kEvInterior))) return rc;
      HIP_TRY(hipEventRecord(s->ev_int, s->s_main));
    } else if (s->sched == 1) {
      // bands(n) then interior(n), both on s_main: the bands run alone
      // briefly and the interior keeps its one-round grid
      HIP_TRY(hipStreamWaitEvent(s->s_main, s->ev_halo, 0));  // halo(n)
      if ((rc = stencil(s->rl_bnd[k], s->pl_bnd[k], s->s_main, kEvBand))) return rc;
      HIP_TRY(hipEventRecord(s->ev_band, s->s_main));
      if ((rc = stencil(s->rl_int[k], s->pl_int[k], s->s_main, kEvInterior))) return rc;
      HIP_TRY(hipEventRecord(s->ev_int, s->s_main));
    } else if (s->sched == 2) {
      // bands(n) on the exchange stream, right before the exchange they feed:
      // the chain bands -> pack -> send/recv -> unpack -> next bands crosses
      // no queue; only interior(n-1) -> bands(n) and bands(n-1) -> interior(n)
      // do (about 11 us per cross-queue wait, profiles/r01/sched)
      HIP_TRY(hipStreamWaitEvent(s->s_main, s->ev_band, 0));  // bands(n-1)
      HIP_TRY(hipStreamWaitEvent(s->s_comm, s->ev_int, 0));   // interior(n-1)
      if ((rc = stencil(s->rl_int[k], s->pl_int[k], s->s_main, kEvInterior))) return rc;
      HIP_TRY(hipEventRecord(s->ev_int, s->s_main));
      if ((rc = stencil(s->rl_bnd[k], s->pl_bnd[k], s->s_comm, kEvBand))) return rc;
      HIP_TRY(hipEventRecord(s->ev_band, s->s_comm));
      if ((rc = enqueue_exchange_timed(s, 1 - k))) return rc;
      s->cur = 1 - k;
      s->t += nsteps;
      return NLH_OK;
    } else {
      HIP_TRY(hipStreamWaitEvent(s->s_main, s->ev_band, 0));  // bands(n-1)
      HIP_TRY(hipStreamWaitEvent(s->s_band, s->ev_int, 0));   // interior(n-1)
      HIP_TRY(hipStreamWaitEvent(s->s_band, s->ev_halo, 0));  // halo(n)
      if ((rc = stencil(s->rl_int[k], s->pl_int[k], s->s_main, kEvInterior))) return rc;
      HIP_TRY(hipEventRecord(s->ev_int, s->s_main));
      if ((rc = stencil(s->rl_bnd[k], s->pl_bnd[k], s->s_band, kEvBand))) return rc;
      HIP_TRY(hipEventRecord(s->ev_band, s->s_band));
    }
    HIP_TRY(hipStreamWaitEvent(s->s_comm, s->ev_band, 0));
    if ((rc = enqueue_exchange_timed(s, 1 - k))) return rc;
  }
  s->cur = 1 - k;
  s->t += nsteps;
  return NLH_OK;
}

int compute_lw(nlh_solver *s) {
  // L_h[W0](x) = sum_disk c*(W0~_j - W0_x)*dh^2; the fast test-mode source is
  // then b = -(2pi st) W0 - ct L_h[W0].  With the two-step kernel (halo 2E)
  // also over the block's E-wide frame: stage 1 computes u^{t+1} there.
  // J = 1 (round 6): from the separable long-double tables (k_lw_sep), the
  // disk sum without the rounding of its N(eps) sequential terms -- at eps
  // 200 that rounding alone put the fast test mode 1.09e-12 of field scale
  // from the compensated oracle at the stable dt (tests/test_gpu_stable_dt.py)
  // -- and O(levels) per node instead of O(N(eps)).  J != 1: the exact
  // per-term order (k_exact's sum)
  const int ext = s->pair ? (int)s->p.eps : 0;
  if (s->d_lty) {
    for (auto &b : s->blocks)
      if (nlh::launch_lw_sep(b.lw_origin(), b.pitch, -ext, -ext, (int)b.r.w + 2 * ext, (int)b.r.h + 2 * ext,
                             (int)b.r.x0, (int)b.r.y0, s->sc, s->sep_nlv, s->sep_lts, s->s_main))
        return fail(NLH_ERR_HIP, "L_h[W0] launch");
    HIP_TRY(hipStreamSynchronize(s->s_main));
    return NLH_OK;
  }
  for (auto &b : s->blocks) {
    double *tmp = b.base[1];
    // the whole buffer: rows above the block as origin() counts them
    if (nlh::launch_fill_w0(tmp, b.pitch, b.xl, (int)b.r.w, (int)b.r.h, (int)((b.rows - b.r.h) / 2), (int)b.r.x0,
                            (int)b.r.y0, s->sc, s->s_main))
      return fail(NLH_ERR_HIP, "fill_w0 launch");
    nlh::RectList rl{};
    rl.nrects = 1;
    nlh::Rect &R = rl.r[0];
    R.u = b.origin(1);
    R.un = b.lw_origin();
    R.pitch = b.pitch;
    R.gx0 = (int32_t)b.r.x0;
    R.gy0 = (int32_t)b.r.y0;
    R.x0 = -ext; R.y0 = -ext; R.x1 = (int)b.r.w + ext; R.y1 = (int)b.r.h + ext;
    R.nstrip = (int)ceil_div(R.x1 - R.x0, 64);
    R.nseg = (int)ceil_div(R.y1 - R.y0, 4);
    rl.nwork = R.nstrip * R.nseg;
    if (nlh::launch_exact_sum(rl, s->sc, s->s_main)) return fail(NLH_ERR_HIP, "L_h[W0] launch");
    HIP_TRY(hipMemsetAsync(b.base[1], 0, b.pitch * b.rows * sizeof(double), s->s_main));
  }
  HIP_TRY(hipStreamSynchronize(s->s_main));
  return NLH_OK;
}

// NLH_TRACE_REPART=1: one JSON line per repartition on stderr with the host
// milliseconds of its phases (diagnostics of the balancing cost)
struct PhaseTrace {
  bool on = false;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
  std::string out;
  void mark(const char *what) {
    if (!on) return;
    const auto t = std::chrono::steady_clock::now();
    char b[64];
    std::snprintf(b, sizeof b, "%s\"%s\": %.3f", out.empty() ? "" : ", ", what,
                  std::chrono::duration<double, std::milli>(t - last).count());
    out += b;
    last = t;
  }
  ~PhaseTrace();
};
thread_local PhaseTrace *g_trace = nullptr;  // the repartition in progress (create_impl marks its phases)
inline void trace_mark(const char *what) {
  if (g_trace) g_trace->mark(what);
}
PhaseTrace::~PhaseTrace() {
  {
    if (on)
      std::fprintf(stderr, "{\"repartition_ms\": {%s}, \"total_ms\": %.3f}\n", out.c_str(),
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
  g_trace = nullptr;
}

// frees every device resource; the communicator too unless keep_comm
void release_impl(nlh_solver *s, bool keep_comm) {
  (void)hipSetDevice(s->device);
  if (s->s_main) (void)hipStreamSynchronize(s->s_main);
  if (s->s_comm) (void)hipStreamSynchronize(s->s_comm);
  if (s->s_band) (void)hipStreamSynchronize(s->s_band);
  if (s->s_copy) (void)hipStreamSynchronize(s->s_copy);
  trace_mark("r_sync");
  for (auto &g : s->graphs) (void)hipGraphExecDestroy(g.exec);
  s->graphs.clear();
  if (s->comm && !keep_comm) ncclCommDestroy(s->comm);
  (void)hipFree(s->snap_dev);
  if (s->snap_host) (void)hipHostFree(s->snap_host);
  if (s->ev_snap_dev) (void)hipEventDestroy(s->ev_snap_dev);
  if (s->ev_snap) (void)hipEventDestroy(s->ev_snap);
  if (s->s_copy) (void)hipStreamDestroy(s->s_copy);
  for (auto &b : s->blocks) {
    (void)hipFree(b.base[0]);
    (void)hipFree(b.base[1]);
    (void)hipFree(b.lw_base);
  }
  trace_mark("r_blocks");
  for (auto &pr : s->peers) {
    (void)hipFree(pr.send);
    (void)hipFree(pr.recv);
  }
  trace_mark("r_peers");
  (void)hipFree(s->d_wt);
  (void)hipFree(s->d_qj);
  (void)hipFree(s->d_ptab);
  (void)hipFree(s->d_lsx);
  (void)hipFree(s->d_lty);
  (void)hipFree(s->d_sxt);
  (void)hipFree(s->d_syt);
  (void)hipFree(s->d_lens);
  (void)hipFree(s->d_part);
  (void)hipFree(s->d_red);
  (void)hipFree(s->stage);
  trace_mark("r_tables");
  for (auto e : s->ev_pool) (void)hipEventDestroy(e);
  if (s->ev_ready) (void)hipEventDestroy(s->ev_ready);
  if (s->ev_halo) (void)hipEventDestroy(s->ev_halo);
  if (s->ev_band) (void)hipEventDestroy(s->ev_band);
  if (s->ev_int) (void)hipEventDestroy(s->ev_int);
  if (s->s_main) (void)hipStreamDestroy(s->s_main);
  if (s->s_comm) (void)hipStreamDestroy(s->s_comm);
  if (s->s_band) (void)hipStreamDestroy(s->s_band);
}

int destroy_impl(nlh_solver *s) {
  if (!s) return NLH_OK;
  release_impl(s, false);
  delete s;
  return NLH_OK;
}

// the streams and events of a solver (swapped between the old and the new
// solver of a repartition)
void swap_queues(nlh_solver *a, nlh_solver *b) {
  std::swap(a->s_main, b->s_main);
  std::swap(a->s_comm, b->s_comm);
  std::swap(a->s_band, b->s_band);
  std::swap(a->ev_ready, b->ev_ready);
  std::swap(a->ev_halo, b->ev_halo);
  std::swap(a->ev_band, b->ev_band);
  std::swap(a->ev_int, b->ev_int);
  std::swap(a->ev_pool, b->ev_pool);
}

// The two-step test-mode pass's separable L_h[W0] (nlh_pair.h OPT & 32768).
// With the reference's zero-extended W0 = sx(x) sy(y) (sx, sy the glibc sin
// values, 0 outside the lattice; sum_local_test, src/2d_nonlocal_serial.cpp:
// 235-252) and the disk as rows dy of half-width len(|dy|):
//   L_h[W0](x, y) = c dh^2 (sum_dy sy(y+dy) Sx_len(|dy|)(x) - N sx(x) sy(y))
//                 = c dh^2 (sum_l Sx'_l(x) Ty_l(y) + sx(x) Z(y)),
// Sx_L = sum_{|dx| <= L} sx(x+dx), Sx'_L = Sx_L - (2L+1) sx (small: no
// cancellation left), Ty_l = the sum of sy(y+dy) over the rows of level l,
// Z = sum_dy (2 len(|dy|) + 1) sy(y+dy) - N sy(y); levels l: the distinct
// len > 0 in order of d (L = 0 rows only enter Z).  Long double sums, c dh^2
// folded into lsx.
int sep_tables(nlh_solver *s, const std::vector<int32_t> &lens) {
  const nlh_params &p = s->p;
  const int E = (int)p.eps;
  std::vector<int> lev;                // = nlh_pair.h pair_sep_level(E, l)
  std::vector<int> lev_of(E + 1, -1);  // half-width -> level index
  for (int d = 0, prev = -1; d <= E; ++d) {
    if (lens[d] > 0 && lens[d] != prev) {
      lev_of[lens[d]] = (int)lev.size();
      lev.push_back(lens[d]);
    }
    prev = lens[d];
  }
  const int nlv = (int)lev.size(), lts = nlh::pair_sep_stride_n(nlv);
  const int64_t ncol = nlh::pair_sep_ncol(E, p.nx);
  // the glibc sin values the kernels use (zero-extended), their long-double
  // prefix sums along x: Sx_L(g) = P(g + L + 1) - P(g - L) in O(1) (round 5
  // summed 2L + 1 sin calls per column and level: O(nx E^2))
  std::vector<long double> sxl(p.nx), syl(p.ny), px(p.nx + 1, 0.0L);
  for (int64_t g = 0; g < p.nx; ++g) sxl[g] = (long double)sin(2 * M_PI * (g * p.dh));
  for (int64_t g = 0; g < p.ny; ++g) syl[g] = (long double)sin(2 * M_PI * (g * p.dh));
  for (int64_t g = 0; g < p.nx; ++g) px[g + 1] = px[g] + sxl[g];
  auto win = [&](int64_t g, int L) {
    return px[std::min<int64_t>(g + L + 1, p.nx)] - px[std::max<int64_t>(g - L, 0)];
  };
  const long double cd = (long double)s->sc.c2d * (long double)s->sc.dh2;
  std::vector<double> lsx((size_t)(nlv + 1) * ncol, 0.0), lty((size_t)(p.ny + 4 * E) * lts, 0.0);
  for (int64_t g = 0; g < p.nx; ++g) {
    const int64_t c = g + 2 * E;
    for (int l = 0; l < nlv; ++l)
      lsx[(size_t)l * ncol + c] = (double)(cd * (win(g, lev[l]) - (2 * lev[l] + 1) * sxl[g]));
    lsx[(size_t)nlv * ncol + c] = (double)(cd * sxl[g]);
  }
  std::vector<long double> ty(nlv);
  for (int64_t y = 0; y < p.ny; ++y) {
    long double z = -(long double)s->disk * syl[y];
    std::fill(ty.begin(), ty.end(), 0.0L);
    for (int d = -E; d <= E; ++d) {
      const int64_t yy = y + d;
      if (yy < 0 || yy >= p.ny) continue;
      const int L = lens[d < 0 ? -d : d];
      z += (2 * L + 1) * syl[yy];
      if (L > 0) ty[lev_of[L]] += syl[yy];
    }
    const size_t r = (size_t)(y + 2 * E) * lts;
    for (int l = 0; l < nlv; ++l) lty[r + l] = (double)ty[l];
    lty[r + nlv] = (double)z;
  }
  HIP_TRY(hipMalloc(&s->d_lsx, lsx.size() * sizeof(double)));
  HIP_TRY(hipMalloc(&s->d_lty, lty.size() * sizeof(double)));
  HIP_TRY(hipMemcpy(s->d_lsx, lsx.data(), lsx.size() * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s->d_lty, lty.data(), lty.size() * sizeof(double), hipMemcpyHostToDevice));
  s->device_bytes += (int64_t)((lsx.size() + lty.size()) * sizeof(double));
  s->sc.lsx = s->d_lsx;
  s->sc.lty = s->d_lty;
  s->sep_nlv = nlv;
  s->sep_lts = lts;
  return NLH_OK;
}

// reuse_comm: an existing communicator over the same ranks (nlh_repartition);
// donor: the solver being repartitioned, whose idle streams and events the
// new one takes over (creating and destroying them was ~13 of ~22 ms per
// repartition, profiles/r05/repart/)
int create_impl(const nlh_params *pin, nlh_solver *s, ncclComm_t reuse_comm = nullptr, nlh_solver *donor = nullptr) {
  const nlh_params &p = *pin;
  if (p.nx <= 0 || p.ny <= 0) return fail(NLH_ERR_ARG, "nx, ny must be positive");
  if (p.eps < 1) return fail(NLH_ERR_ARG, "eps must be >= 1");
  if (p.nx + 2 * p.eps > (1ll << 30) || p.ny + 2 * p.eps > (1ll << 30))
    return fail(NLH_ERR_ARG, "lattice too large for 32-bit node coordinates");
  if (p.nranks < 1 || p.rank < 0 || p.rank >= p.nranks) return fail(NLH_ERR_ARG, "bad rank/nranks");
  const int64_t tx = p.tiles_x > 0 ? p.tiles_x : 1, ty = p.tiles_y > 0 ? p.tiles_y : 1;
  if (p.nx % tx || p.ny % ty) return fail(NLH_ERR_ARG, "tiles_x/tiles_y must divide nx/ny");
  if (p.kernel < NLH_KERNEL_AUTO || p.kernel > NLH_KERNEL_FAST) return fail(NLH_ERR_ARG, "bad kernel");
  if (int rc = check_env()) return rc;
  s->p = p;
  s->p.tiles_x = tx;
  s->p.tiles_y = ty;
  s->p.owner = nullptr;
  s->p.comm_id = nullptr;

  std::string err;
  const int vranks = virtual_ranks(p);
  s->owners = vranks ? vranks : p.nranks;
  if (!nlh::resolve_owner(tx, ty, vranks ? vranks : p.nranks, p.owner, s->owner, err))
    return fail(NLH_ERR_ARG, err);

  // ---- device
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(NLH_ERR_HIP, "no HIP device visible (libnlh has no CPU fallback)");
  if (p.device >= 0) {
    if (p.device >= ndev) return fail(NLH_ERR_ARG, "device ordinal out of range");
    s->device = p.device;
  } else {
    HIP_TRY(hipGetDevice(&s->device));
  }
  HIP_TRY(hipSetDevice(s->device));
  // host waits: nlh_synchronize polls its streams itself (NLH_SYNC unset or
  // 0), so the process-wide host-wait flag of the device stays the
  // application's.  NLH_SYNC=1..4 (A/B diagnostics) sets the flag
  // -- taken only by a device whose context is not yet active; otherwise HIP
  // keeps what it has (error cleared) -- and blocks in hipStreamSynchronize
  s->sync_mode = 0;
  if (const char *v = std::getenv("NLH_SYNC"))
    if (*v) s->sync_mode = std::atoi(v);
  if (s->sync_mode != 0) {
    const unsigned fl = s->sync_mode == 1 ? hipDeviceScheduleYield
                        : s->sync_mode == 2 ? hipDeviceScheduleBlockingSync
                        : s->sync_mode == 3 ? hipDeviceScheduleAuto : hipDeviceScheduleSpin;
    if (hipSetDeviceFlags(fl) != hipSuccess) (void)hipGetLastError();
  }
  if (const char *v = std::getenv("NLH_HOST_PROBE")) s->host_probe = *v && std::atoi(v) != 0;
  if (const char *v = std::getenv("NLH_GRAPH")) s->graph_on = *v && std::atoi(v) != 0;
  if (const char *v = std::getenv("NLH_SEGV_TRACE"))
    if (*v && std::atoi(v) != 0) install_segv_trace();
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, s->device));
  std::snprintf(s->arch, sizeof(s->arch), "%s", prop.gcnArchName);
  s->cus = std::max(1, prop.multiProcessorCount);
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(NLH_ERR_UNSUPPORTED, std::string("libnlh is built for gfx950, device is ") + prop.gcnArchName);

  // ---- kernel choice
  const int E = (int)p.eps;
  Resolved rv;
  if (int rc0 = resolve_config(p, rv)) return rc0;
  const int kern = rv.kernel;
  s->kernel = kern;
  if (const char *r = std::getenv("NLH_FAST_R")) {
    const int v = std::atoi(r);
    s->fast_r = (v == 1 || v == 4) ? v : 2;
  }
  s->fast_r = nlh::fast_lanes_cols(E, s->fast_r);
  s->pair = rv.pair;
  s->wide = rv.wide;
  s->weighted = rv.weighted;
  s->prefix = rv.prefix;
  if (s->prefix) {
    s->prefix_waves = nlh::prefix_rt_waves(E);
    if (!nlh::prefix_rt_waves_ok(E, s->prefix_waves))
      return fail(NLH_ERR_ARG, "NLH_PREFIX_WAVES must be 1, 2, 4, 8 or 16 (its window within the LDS)");
    s->prefix_rows = nlh::prefix_rt_rows(E, s->prefix_waves);
    if (!nlh::prefix_rt_rows_ok(E, s->prefix_rows))
      return fail(NLH_ERR_ARG, "NLH_PREFIX_ROWS must be 32 or 64 (96 or 128 past eps 224)");
  }
  if (const char *fb = std::getenv("NLH_FORCE_BANDS")) s->force_bands = std::atoi(fb) == 1 ? 30 : std::atoi(fb) & 30;
  if (const char *rs = std::getenv("NLH_RCCL_SELF")) s->rccl_self = p.nranks == 1 && std::atoi(rs) != 0;
  if (vranks) s->rccl_self = true;  // virtual owners talk over RCCL to self
  if (const char *ic = std::getenv("NLH_INT_PER_CU")) s->int_per_cu = std::max(0, std::atoi(ic));
  if (const char *sc = std::getenv("NLH_SCHED")) s->sched = std::min(2, std::max(0, std::atoi(sc)));
  int prio_lo = 0, prio_hi = 0;  // NLH_COMM_PRIO=1: exchange + band streams at the highest priority
  if (const char *cp = std::getenv("NLH_COMM_PRIO"))
    if (std::atoi(cp) != 0) HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  if (const char *ps = std::getenv("NLH_PAIR_SPLIT"))
    if (std::atoi(ps) == 1) s->pair_split = 1;  // k_pair_split with 16-slot rings (variant 1)
  if (const char *pc = std::getenv("NLH_PAIR_CU")) s->pair_cu = std::max(1, std::atoi(pc));
  if (const char *pt = std::getenv("NLH_PAIR_TEST")) s->pair_test = std::atoi(pt) == 0 ? 4 : 5;
  if (const char *pp = std::getenv("NLH_PAIR_PRIO")) s->pair_prio = std::atoi(pp);
  s->halo = rv.halo;
  s->plan = nlh::make_plan(p.nx, p.ny, s->halo, tx, ty, s->owner, p.split_tiles == 0);
  s->vranks = vranks;
  s->mine.clear();
  if (vranks)
    for (int v = 0; v < vranks; ++v) s->mine.push_back(v);
  else
    s->mine.push_back((int)p.rank);
  s->ev_acc_owner.assign(s->owners, 0.0);
  trace_mark("c_plan");

  if (donor && donor->s_main) {
    swap_queues(s, donor);
  } else {
    HIP_TRY(hipStreamCreateWithFlags(&s->s_main, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithPriority(&s->s_comm, hipStreamNonBlocking, prio_hi));
    HIP_TRY(hipStreamCreateWithPriority(&s->s_band, hipStreamNonBlocking, prio_hi));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_ready, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_halo, hipEventDisableTiming));
    // the per-pass kernel -> kernel dependencies between the interior and the
    // band streams (one device, device memory only): device-scope release /
    // acquire instead of the system-scope fence.  Round 6, 4096^2 rank proxy
    // (tools/gpu/r6_evfence.sh, profiles/r06/rank_proxy/evfence/): one side
    // 76.4-76.8 against 78.0-79.2 us per pass, three sides 76.2-76.5 against
    // 78.8-79.3 (the main queue's gap at these two events)
    HIP_TRY(hipEventCreateWithFlags(&s->ev_band, hipEventDisableTiming | hipEventDisableSystemFence));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_int, hipEventDisableTiming | hipEventDisableSystemFence));
  }
  HIP_TRY(hipEventRecord(s->ev_band, s->s_main));
  HIP_TRY(hipEventRecord(s->ev_int, s->s_main));
  trace_mark("c_streams");

  // ---- constants and host-computed tables (glibc sin, bit-equal to w())
  std::vector<double> sxt(p.nx + 2 * E), syt(p.ny + 2 * E);
  for (int64_t g = -E; g < p.nx + E; ++g) sxt[g + E] = sin(2 * M_PI * (g * p.dh));
  for (int64_t g = -E; g < p.ny + E; ++g) syt[g + E] = sin(2 * M_PI * (g * p.dh));
  std::vector<int32_t> lens(E + 1);
  s->disk = 0;
  for (int d = 0; d <= E; ++d) lens[d] = (int32_t)(long)sqrt((double)((long)E * E - (long)d * d));
  for (int d = -E; d <= E; ++d) s->disk += 2 * lens[d < 0 ? -d : d] + 1;
  HIP_TRY(hipMalloc(&s->d_sxt, sxt.size() * sizeof(double)));
  HIP_TRY(hipMalloc(&s->d_syt, syt.size() * sizeof(double)));
  HIP_TRY(hipMalloc(&s->d_lens, lens.size() * sizeof(int32_t)));
  HIP_TRY(hipMemcpy(s->d_sxt, sxt.data(), sxt.size() * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s->d_syt, syt.data(), syt.size() * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s->d_lens, lens.data(), lens.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  // c = 2k/(M3 (eps dh)^4) with the code's pi omitted (:76): J = 1 has
  // 2/M3 = 8, the reference's (k*8); J = 1 - r has M3 = 1/20 (tex :159)
  s->sc.c2d = p.influence == NLH_INFLUENCE_LINEAR ? (p.k * 40) / pow(p.eps * p.dh, 4)
                                                  : (p.k * 8) / pow(p.eps * p.dh, 4);
  s->sc.influence = p.influence;
  if (p.influence != NLH_INFLUENCE_CONSTANT || rv.weighted) {
    // J(distance/eps), distance = sqrt(dx^2+dy^2) as the reference's
    // distance() (:224-227); wt in the reference's loop order.  J = 1 tables
    // for k_weighted at eps 33..52
    const bool lin = p.influence == NLH_INFLUENCE_LINEAR;
    auto J = [&](long dx, long dy) {
      return lin ? 1.0 - sqrt((double)(dx * dx + dy * dy)) / (double)p.eps : 1.0;
    };
    std::vector<double> wt, qj((size_t)(E + 1) * (E + 1), 0.0);
    double jsum = 0.0;
    for (long dx = -E; dx <= E; ++dx) {
      const long len = lens[dx < 0 ? -dx : dx];
      for (long dy = -len; dy <= len; ++dy) {
        wt.push_back(J(dx, dy) * s->sc.c2d);
        jsum += J(dx, dy);
      }
    }
    for (long dx = 0; dx <= E; ++dx)
      for (long dy = 0; dy <= lens[dx]; ++dy) qj[(size_t)(dx * (E + 1) + dy)] = J(dx, dy);
    HIP_TRY(hipMalloc(&s->d_wt, wt.size() * sizeof(double)));
    HIP_TRY(hipMalloc(&s->d_qj, qj.size() * sizeof(double)));
    HIP_TRY(hipMemcpy(s->d_wt, wt.data(), wt.size() * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->d_qj, qj.data(), qj.size() * sizeof(double), hipMemcpyHostToDevice));
    s->sc.wt = s->d_wt;
    s->sc.qj = s->d_qj;
    s->sc.jsum = jsum;
  }
  s->sc.dh2 = p.dh * p.dh;
  s->sc.dt = p.dt;
  s->sc.alpha = s->sc.c2d * s->sc.dh2 * p.dt;
  s->sc.nf = (double)s->disk;
  s->sc.kc = (s->pair || s->wide || s->prefix) ? 1.0 / s->sc.alpha - s->sc.nf : 0.0;
  if (s->prefix) {
    std::vector<int32_t> tab(2 * (size_t)nlh::prefix_rt_table_size(E, s->prefix_rows));
    nlh::prefix_rt_table(E, s->prefix_rows, lens.data(), tab.data());
    HIP_TRY(hipMalloc(&s->d_ptab, tab.size() * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(s->d_ptab, tab.data(), tab.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  if (kern == NLH_KERNEL_FAST && p.test && p.influence == NLH_INFLUENCE_CONSTANT) {  // compute_lw's L_h[W0]
    int rc2 = sep_tables(s, lens);
    if (rc2) return rc2;
  }
  s->sc.sxt = s->d_sxt;
  s->sc.syt = s->d_syt;
  s->sc.lens = s->d_lens;
  s->sc.nx = p.nx;
  s->sc.ny = p.ny;
  s->sc.E = E;
  set_time(s, 0);
  trace_mark("c_tables");

  // ---- local blocks, padded (see nlh_device.h)
  const int64_t XL = round_up(s->halo, 8);
  int64_t pitch_pad = 0;  // extra doubles per row (layout experiments, NLH_PITCH_PAD)
  if (const char *pp = std::getenv("NLH_PITCH_PAD")) pitch_pad = 2 * (std::max(0, std::atoi(pp)) / 2);
  for (size_t i = 0; i < s->plan.blocks.size(); ++i) {
    const auto &bd = s->plan.blocks[i];
    if (!vranks && bd.rank != p.rank) continue;  // virtual ranks: this process runs every block
    LocalBlock b;
    b.plan_index = (int)i;
    b.owner = bd.rank;
    b.r = bd.r;
    b.xl = (int32_t)XL;
    // whole 256-column strips stay in bounds; the pair kernel's last strip
    // stages up to column w + 127
    // (k_prefix_rt stages 64 NV <= 512 columns from x0 - E of its last strip,
    // k_prefix_rtc 512-column chunks: prefix_rt_window)
    const int64_t right = std::max({round_up(b.r.w, 256) + XL, s->pair ? b.r.w + 128 : (int64_t)0,
                                    s->prefix ? round_up(b.r.w, 64) + nlh::prefix_rt_window(E, s->prefix_waves) : (int64_t)0});
    b.pitch = round_up(XL + right, 8) + pitch_pad;
    // pair passes: padding rows beyond the halo rows, above and below, that
    // k_pair_split's tail row DMAs read instead of clamping (nlh_pair.h)
    b.rows = b.r.h + 2 * (s->halo + (s->pair ? nlh::pair_pad_rows() : 0));
    b.L = b.r.x0 > 0 || (s->force_bands & 2);
    b.Rr = b.r.x0 + b.r.w < p.nx || (s->force_bands & 4);
    b.T = b.r.y0 > 0 || (s->force_bands & 8);
    b.B = b.r.y0 + b.r.h < p.ny || (s->force_bands & 16);
    const size_t bytes = (size_t)(b.pitch * b.rows) * sizeof(double);
    // zeroed on s_main (a non-blocking stream: a null-stream hipMemset is not
    // ordered before work on it), and waited for below, before anything --
    // test_init, set_field, a repartition's tile copies -- writes the blocks
    for (int k = 0; k < 2; ++k) {
      HIP_TRY(hipMalloc(&b.base[k], bytes));
      HIP_TRY(hipMemsetAsync(b.base[k], 0, bytes, s->s_main));
      s->device_bytes += (int64_t)bytes;
    }
    if (kern == NLH_KERNEL_FAST && p.test) {
      HIP_TRY(hipMalloc(&b.lw_base, bytes));
      HIP_TRY(hipMemsetAsync(b.lw_base, 0, bytes, s->s_main));
      s->device_bytes += (int64_t)bytes;
    }
    s->blocks.push_back(b);
  }
  HIP_TRY(hipStreamSynchronize(s->s_main));
  trace_mark("c_blocks");

  s->exchange_planned = !s->plan.pieces.empty() || s->force_bands != 0;
  int rc = build_rectlists(s, 0);
  if (rc) return rc;
  if (s->pair && (rc = build_rectlists(s, 1))) return rc;
  trace_mark("c_rectlists");

  // ---- RCCL communicator and exchange plan
  if (reuse_comm) {
    s->comm = reuse_comm;
  } else if (p.nranks > 1) {
    if (!p.comm_id) return fail(NLH_ERR_ARG, "nranks > 1 requires comm_id");
    ncclUniqueId id;
    static_assert(sizeof(ncclUniqueId) == NLH_COMM_ID_BYTES, "unique id size");
    std::memcpy(&id, p.comm_id, sizeof(id));
    rc = comm_init_bounded(&s->comm, p.nranks, id, p.rank, s->device);
    if (rc) return rc;
  } else if (s->rccl_self) {
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    NCCL_TRY(ncclCommInitRank(&s->comm, 1, id, 0));
  }
  if (s->comm) {
    // the communicator's own view of the job: a real run must see every rank
    // (a mis-launched job fails here instead of exchanging with the wrong peers)
    int cn = 0, cr = -1;
    NCCL_TRY(ncclCommCount(s->comm, &cn));
    NCCL_TRY(ncclCommUserRank(s->comm, &cr));
    s->comm_nranks = cn;
    s->comm_rank = cr;
    const int want_n = p.nranks > 1 ? (int)p.nranks : 1, want_r = p.nranks > 1 ? (int)p.rank : 0;
    if (cn != want_n || cr != want_r)
      return fail(NLH_ERR_RCCL, "RCCL communicator has " + std::to_string(cn) + " ranks (this one " +
                                    std::to_string(cr) + "), expected " + std::to_string(want_n) + " (rank " +
                                    std::to_string(want_r) + ")");
  }
  trace_mark("c_comm");
  rc = build_exchange(s);
  if (rc) return rc;
  trace_mark("c_exchange");
  if (s->exchange && !s->comm && !s->peers.empty())
    return fail(NLH_ERR_STATE, "internal: peers without communicator");

  // ---- norm scratch
  int tot = 0;
  for (auto &b : s->blocks) {
    s->part_off.push_back(tot);
    tot += nlh::norm_workgroups((int)b.r.w, (int)b.r.h);
  }
  s->part_total = tot;
  HIP_TRY(hipMalloc(&s->d_part, std::max(tot, 1) * sizeof(nlh::NormPartial)));
  HIP_TRY(hipMalloc(&s->d_red, 2 * sizeof(double)));

  if (kern == NLH_KERNEL_FAST && p.test) {
    rc = compute_lw(s);
    if (rc) return rc;
  }
  return NLH_OK;
}

// ncclCommInitRank with a bounded wait (a first multi-GPU
// run that hangs in the rendezvous must exit with a diagnosis, not block until
// the job's time limit).  The init runs on a helper thread (same device); the
// caller waits up to NLH_COMM_INIT_TIMEOUT seconds (default 300).  On a
// timeout the helper stays blocked inside RCCL and is detached -- its state is
// shared, so it never writes to freed memory -- and nlh_create fails with
// NLH_ERR_RCCL "... timed out"; the process is expected to exit (bench.py
// prints its error line and does).  The communicator itself stays a blocking
// one: no call after the init changes.
struct CommInit {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  ncclResult_t r = ncclInternalError;
  ncclComm_t comm = nullptr;
};

int comm_init_bounded(ncclComm_t *out, int nranks, const ncclUniqueId &id, int rank, int device) {
  int timeout_s = 300;
  if (const char *v = std::getenv("NLH_COMM_INIT_TIMEOUT"))
    if (*v) timeout_s = std::atoi(v);
  auto st = std::make_shared<CommInit>();
  std::thread th([st, nranks, id, rank, device] {
    ncclComm_t c = nullptr;
    ncclResult_t r = hipSetDevice(device) == hipSuccess ? ncclCommInitRank(&c, nranks, id, rank) : ncclUnhandledCudaError;
    std::lock_guard<std::mutex> lk(st->m);
    st->comm = c;
    st->r = r;
    st->done = true;
    st->cv.notify_all();
  });
  std::unique_lock<std::mutex> lk(st->m);
  const bool ok = st->cv.wait_for(lk, std::chrono::seconds(timeout_s), [&] { return st->done; });
  lk.unlock();
  if (!ok) {
    th.detach();
    return fail(NLH_ERR_RCCL, "ncclCommInitRank (rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                                  ") timed out after " + std::to_string(timeout_s) +
                                  " s (NLH_COMM_INIT_TIMEOUT): a peer rank never joined the communicator");
  }
  th.join();
  if (st->r != ncclSuccess)
    return fail(NLH_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(st->r));
  *out = st->comm;
  return NLH_OK;
}

// A point-to-point message of cnt doubles, posted (inside the caller's group)
// as in-order chunks of at most kP2PChunk doubles (256 MiB).  With RCCL
// 2.27.7 on MI355X a single 1.5 GiB send/recv to self (three 8192^2 tiles of a
// repartition) delivered only its first 512 MiB and a 3 GiB root gather
// arrived corrupted, in every run; 0.5 and 1 GiB messages arrived whole
// (profiles/r04/{fourth,fifth,sixth}: diag_8192.log, the large-move test).
// The chunks match pairwise in order on both sides.
constexpr size_t kP2PChunk = size_t(1) << 25;
// a repartition's staging buffer stays with the solver for the next one up
// to this size (tile moves of a few tiles; larger ones are freed after use)
constexpr size_t kStageKeepBytes = size_t(2) << 30;
bool p2p(bool send, double *buf, size_t cnt, int peer, ncclComm_t comm, hipStream_t st) {
  for (size_t o = 0; o < cnt; o += kP2PChunk) {
    const size_t c = std::min(kP2PChunk, cnt - o);
    if ((send ? ncclSend(buf + o, c, ncclDouble, peer, comm, st) : ncclRecv(buf + o, c, ncclDouble, peer, comm, st)) !=
        ncclSuccess)
      return false;
  }
  return true;
}

// the plan block holding global node (x, y): its rank and local block index
void locate(const nlh_solver *s, int64_t x, int64_t y, int &rank, int &local) {
  rank = -1;
  local = -1;
  for (size_t b = 0; b < s->plan.blocks.size(); ++b) {
    const nlh::GRect &r = s->plan.blocks[b].r;
    if (x < r.x0 || x >= r.x0 + r.w || y < r.y0 || y >= r.y0 + r.h) continue;
    rank = s->plan.blocks[b].rank;
    for (size_t j = 0; j < s->blocks.size(); ++j)
      if (s->blocks[j].plan_index == (int)b) local = (int)j;
    return;
  }
}

double *tile_ptr(const nlh_solver *s, int local, int k, int64_t x0, int64_t y0) {
  const LocalBlock &b = s->blocks[local];
  return b.origin(k) + (y0 - b.r.y0) * b.pitch + (x0 - b.r.x0);
}

bool runs(const nlh_solver *s, int rank) {
  return std::find(s->mine.begin(), s->mine.end(), rank) != s->mine.end();
}

// The new solver is built beside the old one (both live until the tiles have
// moved), plus one staging copy of the moving tiles on each side: check the
// device's free memory against that before allocating anything, so a
// rebalance that does not fit leaves the run as it was (NLH_ERR_NOMEM; the
// distributed driver then skips that rebalance).  Every rank of a real
// multi-rank run takes the same decision (minimum over ranks), so no rank
// waits in a tile send that the others skip.
int repartition_fits(nlh_solver *s, const std::vector<int32_t> &own) {
  int64_t tiles_old = 0, tiles_new = 0, moving = 0;
  for (size_t i = 0; i < own.size(); ++i) {
    const bool ro = runs(s, s->owner[i]), rn = runs(s, own[i]);
    tiles_old += ro;
    tiles_new += rn;
    if (own[i] != s->owner[i]) moving += (int64_t)ro + (int64_t)rn;
  }
  const int64_t tile_bytes = (s->p.nx / s->p.tiles_x) * (s->p.ny / s->p.tiles_y) * (int64_t)sizeof(double);
  const double scale = tiles_old > 0 ? (double)tiles_new / (double)tiles_old : 1.0;
  // staging: the kept buffer (stage_cap, already allocated, so not in the free
  // memory) covers that much of the moving tiles; repartition_impl frees it
  // before allocating a larger one (round 5 counted it twice)
  const double stage_new = std::max(0.0, (double)(moving * tile_bytes) - (double)s->stage_cap * sizeof(double));
  const double need = (double)s->device_bytes * scale * 1.05 + stage_new + 64.0 * (1 << 20);
  size_t free_b = 0, total_b = 0;
  // a local failure votes "does not fit" but still joins the all-reduce below:
  // returning early here would leave the other ranks waiting in it
  double ok = hipMemGetInfo(&free_b, &total_b) == hipSuccess && (double)free_b >= need ? 1.0 : 0.0;
  if (s->comm && !s->vranks && s->p.nranks > 1) {
    // the vote travels in the solver's own reduction scratch (d_red): the
    // check allocates nothing
    int st = NLH_OK;
    // a zero vote first: if the upload below fails, this rank still
    // joins the all-reduce with "does not fit", never with whatever the scratch
    // held last (an L2 partial that can be >= 1)
    if (hipMemsetAsync(s->d_red, 0, sizeof(double), s->s_comm) != hipSuccess) {
      st = fail(NLH_ERR_HIP, "repartition memory check clear");
      ok = 0.0;
    }
    if (st == NLH_OK && ok == 1.0 &&
        hipMemcpyAsync(s->d_red, &ok, sizeof(double), hipMemcpyHostToDevice, s->s_comm) != hipSuccess) {
      st = fail(NLH_ERR_HIP, "repartition memory check upload");
      ok = 0.0;
    }
    // every rank reaches this collective whatever happened above
    if (ncclAllReduce(s->d_red, s->d_red, 1, ncclDouble, ncclMin, s->comm, s->s_comm) != ncclSuccess && st == NLH_OK)
      st = fail(NLH_ERR_RCCL, "repartition memory check all-reduce");
    double agreed = 0.0;
    if (st == NLH_OK && hipMemcpyAsync(&agreed, s->d_red, sizeof(double), hipMemcpyDeviceToHost, s->s_comm) != hipSuccess)
      st = fail(NLH_ERR_HIP, "repartition memory check download");
    if (hipStreamSynchronize(s->s_comm) != hipSuccess && st == NLH_OK) st = fail(NLH_ERR_HIP, "repartition sync");
    if (st) return st;
    ok = agreed;
  }
  if (ok < 1.0) {
    char buf[200];
    std::snprintf(buf, sizeof buf, "repartition needs ~%.0f MiB of device memory, %.0f MiB free (on this or another rank); "
                  "the solver is unchanged", need / (1 << 20), (double)free_b / (1 << 20));
    return fail(NLH_ERR_NOMEM, buf);
  }
  return NLH_OK;
}

// rebuild the solver for a new tile -> owner map, moving the tiles that
// change rank over RCCL (src/2d_nonlocal_distributed.cpp:937-944).  Per
// (virtual) rank pair A -> B the moving tiles travel in tile order as one
// message; with virtual ranks A's message goes through RCCL to self into B's
// staging buffer, as a real run's would to rank B.
int repartition_impl(nlh_solver *s, const std::vector<int32_t> &own) {
  if (s->snap_pending) return fail(NLH_ERR_STATE, "a snapshot is in flight (call nlh_snapshot_wait)");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_main));
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  HIP_TRY(hipStreamSynchronize(s->s_band));
  if (own == s->owner) return NLH_OK;
  PhaseTrace tr;
  if (const char *e = std::getenv("NLH_TRACE_REPART")) tr.on = std::atoi(e) != 0;
  if (tr.on) g_trace = &tr;
  nlh_params p = s->p;
  p.owner = own.data();
  p.comm_id = nullptr;
  if ((rc = repartition_fits(s, own))) return rc;
  tr.mark("fits_vote");
  nlh_solver *n = new nlh_solver();
  rc = create_impl(&p, n, s->comm, s);
  tr.mark("create");
  if (rc) {
    const std::string keep = g_err;
    n->comm = nullptr;  // still the caller's
    if (!s->s_main) swap_queues(s, n);  // the old solver's streams back
    destroy_impl(n);
    g_err = keep;
    return rc;
  }
  const int64_t tw = p.nx / p.tiles_x, th = p.ny / p.tiles_y;
  struct Mv {
    int64_t x0, y0;
    int src, dst;  // local block indices in s (source) and n (destination)
  };
  std::vector<Mv> local;
  // (sender, receiver) -> tiles in tile order; sends hold the sender's side,
  // recvs the receiver's
  std::map<std::pair<int, int>, std::vector<Mv>> sends, recvs;
  for (int64_t i = 0; i < p.tiles_x * p.tiles_y; ++i) {
    const int64_t x0 = (i % p.tiles_x) * tw, y0 = (i / p.tiles_x) * th;
    int ro, lo, rn, ln;
    locate(s, x0, y0, ro, lo);
    locate(n, x0, y0, rn, ln);
    if (ro == rn && runs(s, ro)) {
      local.push_back({x0, y0, lo, ln});
      continue;
    }
    if (runs(s, ro)) sends[{ro, rn}].push_back({x0, y0, lo, -1});
    if (runs(s, rn)) recvs[{ro, rn}].push_back({x0, y0, -1, ln});
  }
  const size_t tb = (size_t)(tw * th);
  const size_t pitch_b = (size_t)tw * sizeof(double);
  int status = NLH_OK;
  // staging: one buffer for every pack and receive, the old solver's when it
  // is large enough (kept across repartitions up to kStageKeepBytes)
  size_t need = 0;
  for (auto &kv : sends) need += kv.second.size() * tb;
  for (auto &kv : recvs) need += kv.second.size() * tb;
  if (need > s->stage_cap) {
    (void)hipFree(s->stage);
    s->stage = nullptr;
    s->stage_cap = 0;
    if (hipMalloc(&s->stage, need * sizeof(double)) == hipSuccess) s->stage_cap = need;
    else s->stage = nullptr;
  }
  size_t stage_used = 0;
  auto stage = [&](size_t ntiles) -> double * {
    if (!s->stage || stage_used + ntiles * tb > s->stage_cap) return nullptr;
    double *b = s->stage + stage_used;
    stage_used += ntiles * tb;
    return b;
  };
  hipStream_t st = n->s_main;
  for (const Mv &m : local) {
    if (hipMemcpy2DAsync(tile_ptr(n, m.dst, 0, m.x0, m.y0), n->blocks[m.dst].pitch * sizeof(double),
                         tile_ptr(s, m.src, s->cur, m.x0, m.y0), s->blocks[m.src].pitch * sizeof(double),
                         pitch_b, th, hipMemcpyDeviceToDevice, st) != hipSuccess)
      status = fail(NLH_ERR_HIP, "repartition local copy");
  }
  std::map<std::pair<int, int>, double *> sbuf, rbuf;
  for (auto &kv : sends) {
    double *b = stage(kv.second.size());
    if (!b) { status = fail(NLH_ERR_HIP, "repartition staging"); break; }
    sbuf[kv.first] = b;
    for (size_t j = 0; j < kv.second.size() && status == NLH_OK; ++j) {
      const Mv &m = kv.second[j];
      if (hipMemcpy2DAsync(b + j * tb, pitch_b, tile_ptr(s, m.src, s->cur, m.x0, m.y0),
                           s->blocks[m.src].pitch * sizeof(double), pitch_b, th, hipMemcpyDeviceToDevice,
                           st) != hipSuccess)
        status = fail(NLH_ERR_HIP, "repartition pack");
    }
  }
  for (auto &kv : recvs) {
    if (status != NLH_OK) break;
    double *b = stage(kv.second.size());
    if (!b) { status = fail(NLH_ERR_HIP, "repartition staging"); break; }
    rbuf[kv.first] = b;
  }
  if (status == NLH_OK && (!sends.empty() || !recvs.empty())) {
    if (!n->comm) {
      status = fail(NLH_ERR_STATE, "internal: tiles change rank without a communicator");
    } else {
      bool ok = ncclGroupStart() == ncclSuccess;
      if (s->vranks) {
        for (auto &kv : sends) {  // A -> B: A's staged tiles into B's staging buffer, over RCCL to self
          const size_t cnt = kv.second.size() * tb;
          ok = ok && recvs.count(kv.first) && recvs[kv.first].size() == kv.second.size();
          for (size_t o = 0; ok && o < cnt; o += kP2PChunk) {
            const size_t c = std::min(kP2PChunk, cnt - o);
            ok = p2p(true, sbuf[kv.first] + o, c, 0, n->comm, st) && p2p(false, rbuf[kv.first] + o, c, 0, n->comm, st);
          }
        }
      } else {
        for (auto &kv : sends) ok = ok && p2p(true, sbuf[kv.first], kv.second.size() * tb, kv.first.second, n->comm, st);
        for (auto &kv : recvs) ok = ok && p2p(false, rbuf[kv.first], kv.second.size() * tb, kv.first.first, n->comm, st);
      }
      ok = (ncclGroupEnd() == ncclSuccess) && ok;
      if (!ok) status = fail(NLH_ERR_RCCL, "repartition send/recv");
    }
  }
  for (auto &kv : recvs) {
    if (status != NLH_OK) break;
    for (size_t j = 0; j < kv.second.size(); ++j) {
      const Mv &m = kv.second[j];
      if (hipMemcpy2DAsync(tile_ptr(n, m.dst, 0, m.x0, m.y0), n->blocks[m.dst].pitch * sizeof(double),
                           rbuf[kv.first] + j * tb, pitch_b, pitch_b, th, hipMemcpyDeviceToDevice,
                           st) != hipSuccess)
        status = fail(NLH_ERR_HIP, "repartition unpack");
    }
  }
  tr.mark("enqueue_moves");
  if (hipStreamSynchronize(st) != hipSuccess && status == NLH_OK) status = fail(NLH_ERR_HIP, "repartition sync");
  tr.mark("moves");
  if (s->stage_cap * sizeof(double) > kStageKeepBytes) {
    (void)hipFree(s->stage);
    s->stage = nullptr;
    s->stage_cap = 0;
  }
  tr.mark("free_staging");
  if (status != NLH_OK) {
    const std::string keep = g_err;
    n->comm = nullptr;
    swap_queues(s, n);  // the old solver's streams back
    destroy_impl(n);
    g_err = keep;
    return status;
  }
  std::swap(n->stage, s->stage);  // the staging buffer lives on in n
  std::swap(n->stage_cap, s->stage_cap);
  n->t = s->t;
  n->cur = 0;
  n->halo_fresh = false;
  n->timing = s->timing;
  n->launch_overhead_ms = s->launch_overhead_ms;
  n->pair_overhead_ms = s->pair_overhead_ms;
  release_impl(s, true);  // the communicator lives on in n (and the streams: s holds none now)
  tr.mark("release_old");
  *s = std::move(*n);
  delete n;  // moved-from shell: its resources now belong to s
  return NLH_OK;
}

// one completed pair into the running totals; busy pairs lose the measured
// empty-launch overhead of each launch they bracket
int fold_pair(nlh_solver *s, size_t p) {
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, s->ev_pool[2 * p], s->ev_pool[2 * p + 1]));
  const EvMeta &m = s->ev_meta[p];
  double v = ms;
  if (m.launches > 0) v = std::max(0.0, v - s->pair_overhead_ms - m.launches * s->launch_overhead_ms);
  s->ev_acc_kind[m.kind] += v;
  if (m.owner >= 0 && m.owner < (int)s->ev_acc_owner.size()) s->ev_acc_owner[m.owner] += v;
  return NLH_OK;
}

// Fold recorded event pairs into the running totals and recycle their events.
// drain: wait for every stream first and fold all.  Otherwise (the pool is
// full inside a long run) wait only until the older half of the pairs has
// completed and fold the pairs that have, keeping the rest in flight: the
// host does not drain the GPU's queue.
int fold_events(nlh_solver *s, bool drain) {
  const size_t npairs = s->ev_meta.size();
  if (drain) {
    HIP_TRY(hipStreamSynchronize(s->s_main));
    HIP_TRY(hipStreamSynchronize(s->s_comm));
    HIP_TRY(hipStreamSynchronize(s->s_band));
  } else if (npairs > 0) {
    // the newest closed pair of the older half
    for (size_t p = npairs / 2 + 1; p-- > 0;)
      if (!s->ev_meta[p].open) {
        HIP_TRY(hipEventSynchronize(s->ev_pool[2 * p + 1]));
        break;
      }
  }
  size_t keep = 0;
  for (size_t p = 0; p < npairs; ++p) {
    if (s->ev_meta[p].open || !drain) {
      const hipError_t q = s->ev_meta[p].open ? hipErrorNotReady : hipEventQuery(s->ev_pool[2 * p + 1]);
      if (q == hipErrorNotReady) {  // still running (or open): move it to the front, fold later
        std::swap(s->ev_pool[2 * keep], s->ev_pool[2 * p]);
        std::swap(s->ev_pool[2 * keep + 1], s->ev_pool[2 * p + 1]);
        s->ev_meta[keep++] = s->ev_meta[p];
        continue;
      }
      if (q != hipSuccess) return fail(NLH_ERR_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
    }
    if (int rc = fold_pair(s, p)) return rc;
  }
  s->ev_used = 2 * keep;
  s->ev_meta.resize(keep);
  return NLH_OK;
}

// ---- HIP graphs of production passes (NLH_GRAPH=1)
// A run of g passes is captured once per (g, start parity) and replayed with
// one hipGraphLaunch on s_main.  The kernels and their arguments are the
// ungraphed ones: bitwise equal fields.  Production mode only (test mode's
// per-step source constants are kernel arguments), kernel timing 0 / 1 only,
// and only for single-stream solvers (no exchange).  Measured on MI355X with
// ROCm 7.2 (profiles/r06/graph): a graph launch costs
// the host about what its nodes' direct launches cost once side streams are
// in it (C3's 8 virtual ranks: 86 -> 73 us of enqueue per pass), and graphs
// with the exchange on side streams -- captured with fork / join events, with
// or without grouped ncclSend / ncclRecv inside -- killed the process with
// SIGSEGV inside nlh_run in 3 of 4 whole-suite runs (never alone, never
// under pytest -s); on one stream (one block) it halves nlh_run's enqueue
// (32 -> 13-18 us for 10 passes) and changes nothing the GPU sees.  So the
// exchange passes stay ungraphed and graphs stay an option, off by default.
constexpr int kGraphMaxPasses = 16;

int graph_passes(const nlh_solver *s, int64_t passes_left) {
  if (!s->graph_on || s->p.test || (s->timing != 0 && s->timing != 1)) return 0;
  if (s->exchange) return 0;
  int g = 0;
  for (int c = 2; c <= kGraphMaxPasses && c <= passes_left; c *= 2) g = c;
  return g;
}

int capture_graph(nlh_solver *s, int g, int spp, hipGraphExec_t *out) {
  const int64_t t0 = s->t, steps0 = s->timed_steps, passes0 = s->timed_passes;
  const int cur0 = s->cur;
  HIP_TRY(hipStreamBeginCapture(s->s_main, hipStreamCaptureModeRelaxed));
  int rc = NLH_OK;
  for (int j = 0; j < g && rc == NLH_OK; ++j) rc = enqueue_step(s, spp);
  hipGraph_t graph = nullptr;
  const hipError_t ec = hipStreamEndCapture(s->s_main, &graph);
  s->t = t0;
  s->cur = cur0;
  s->timed_steps = steps0;
  s->timed_passes = passes0;
  if (rc) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  if (ec != hipSuccess) return fail(NLH_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ec));
  const hipError_t ei = hipGraphInstantiate(out, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ei != hipSuccess) return fail(NLH_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
  return NLH_OK;
}

// g passes from the current step: the captured graph (captured now if new)
int launch_graph(nlh_solver *s, int g, int spp) {
  nlh_solver::Graph *ge = nullptr;
  for (auto &x : s->graphs)
    if (x.passes == g && x.k == s->cur) ge = &x;
  if (!ge) {
    nlh_solver::Graph n;
    n.passes = g;
    n.k = s->cur;
    if (int rc = capture_graph(s, g, spp, &n.exec)) return rc;
    s->graphs.push_back(n);
    ge = &s->graphs.back();
  }
  HIP_TRY(hipGraphLaunch(ge->exec, s->s_main));
  if (g & 1) s->cur = 1 - s->cur;
  s->t += (int64_t)g * spp;
  if (s->timing) {
    s->timed_steps += (int64_t)g * spp;
    s->timed_passes += g;
  }
  return NLH_OK;
}

// wait for a stream by polling it (NLH_SYNC 0): no host-wait flag of the
// device is needed and the host sees the GPU finish within a query's time.
// watch: record when the last nlh_run's end event is first seen complete
// (nlh_host_time).  Past kPollNs the wait blocks in HIP instead, so long runs
// do not hold a core
int poll_stream(nlh_solver *s, hipStream_t st, bool watch) {
  constexpr int64_t kPollNs = 200000000;  // 0.2 s
  const int64_t t0 = now_ns();
  watch = watch && s->h_e1 != nullptr && s->h_end_seen < 0;
  for (;;) {
    if (watch) {
      const hipError_t q = hipEventQuery(s->h_e1);
      if (q == hipSuccess) {
        s->h_end_seen = now_ns();
        watch = false;
      } else if (q != hipErrorNotReady) {
        return fail(NLH_ERR_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
      }
    }
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) return fail(NLH_ERR_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(q));
    if (now_ns() - t0 > kPollNs) {
      HIP_TRY(hipStreamSynchronize(st));
      break;
    }
  }
  if (watch && hipEventQuery(s->h_e1) == hipSuccess) s->h_end_seen = now_ns();
  return NLH_OK;
}

// busy milliseconds of each (virtual) rank this process runs since busy
// timing was enabled (index = rank; ranks run elsewhere stay 0)
int owner_busy(nlh_solver *s, std::vector<double> &ms) {
  if (int rc = fold_events(s, true)) return rc;
  ms = s->ev_acc_owner;
  return NLH_OK;
}

}  // namespace

extern "C" {

int nlh_abi_version(void) { return NLH_ABI_VERSION; }

const char *nlh_last_error(void) { return g_err.c_str(); }

int nlh_comm_unique_id(uint8_t id[NLH_COMM_ID_BYTES]) {
  if (!id) return fail(NLH_ERR_ARG, "null id");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(NLH_ERR_HIP, "no HIP device visible (libnlh has no CPU fallback)");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return NLH_OK;
}

int nlh_create(const nlh_params *p, nlh_solver **out) {
  if (!p || !out) return fail(NLH_ERR_ARG, "null argument");
  *out = nullptr;
  nlh_solver *s = new nlh_solver();
  int rc = create_impl(p, s);
  if (rc != NLH_OK) {
    const std::string keep = g_err;
    destroy_impl(s);
    g_err = keep;
    return rc;
  }
  *out = s;
  return NLH_OK;
}

int nlh_destroy(nlh_solver *s) { return destroy_impl(s); }

int nlh_init_test(nlh_solver *s) {
  if (!s) return fail(NLH_ERR_ARG, "null solver");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  s->cur = 0;
  s->t = 0;
  s->halo_fresh = false;
  for (auto &b : s->blocks)
    if (nlh::launch_init_test(b.origin(0), b.pitch, (int)b.r.w, (int)b.r.h, (int)b.r.x0,
                              (int)b.r.y0, s->sc, s->s_main))
      return fail(NLH_ERR_HIP, "init launch");
  HIP_TRY(hipStreamSynchronize(s->s_main));
  return NLH_OK;
}

int nlh_set_field(nlh_solver *s, const double *u) {
  if (!s || !u) return fail(NLH_ERR_ARG, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  HIP_TRY(hipStreamSynchronize(s->s_main));
  s->cur = 0;
  s->t = 0;
  s->halo_fresh = false;
  for (auto &b : s->blocks)
    HIP_TRY(hipMemcpy2D(b.origin(0), b.pitch * sizeof(double), u + b.r.y0 * s->p.nx + b.r.x0,
                        s->p.nx * sizeof(double), b.r.w * sizeof(double), b.r.h,
                        hipMemcpyHostToDevice));
  return NLH_OK;
}

int nlh_get_field(nlh_solver *s, double *u) {
  if (!s || !u) return fail(NLH_ERR_ARG, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  HIP_TRY(hipStreamSynchronize(s->s_main));
  for (auto &b : s->blocks)
    HIP_TRY(hipMemcpy2D(u + b.r.y0 * s->p.nx + b.r.x0, s->p.nx * sizeof(double), b.origin(s->cur),
                        b.pitch * sizeof(double), b.r.w * sizeof(double), b.r.h,
                        hipMemcpyDeviceToHost));
  return NLH_OK;
}

int nlh_gather_field(nlh_solver *s, int32_t root, double *u) {
  if (!s) return fail(NLH_ERR_ARG, "null solver");
  if (root < 0 || root >= s->owners) return fail(NLH_ERR_ARG, "bad root");
  const bool at_root = runs(s, root);
  if (at_root && !u) return fail(NLH_ERR_ARG, "root needs an output array");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  HIP_TRY(hipStreamSynchronize(s->s_main));
  // the root's own blocks straight to the host
  if (at_root)
    for (auto &b : s->blocks)
      if (b.owner == root)
        HIP_TRY(hipMemcpy2D(u + b.r.y0 * s->p.nx + b.r.x0, s->p.nx * sizeof(double), b.origin(s->cur),
                            b.pitch * sizeof(double), b.r.w * sizeof(double), b.r.h, hipMemcpyDeviceToHost));
  if (!s->comm) return NLH_OK;
  // every other (virtual) rank ships its blocks packed in plan order; the
  // root unpacks by the plan.  With virtual ranks each one's message travels
  // over RCCL to self, as a real rank's would to the root
  std::vector<int64_t> count(s->owners, 0);
  for (auto &b : s->plan.blocks) count[b.rank] += b.r.w * b.r.h;
  int64_t maxc = 1;
  for (int r = 0; r < s->owners; ++r) maxc = std::max(maxc, count[r]);
  double *sbuf = nullptr, *rbuf = nullptr;
  HIP_TRY(hipMalloc(&sbuf, maxc * sizeof(double)));
  if (hipMalloc(&rbuf, maxc * sizeof(double)) != hipSuccess) {
    (void)hipFree(sbuf);
    return fail(NLH_ERR_HIP, "gather buffer");
  }
  int status = NLH_OK;
  auto pack = [&](int r) {
    int64_t off = 0;
    for (auto &b : s->blocks) {
      if (b.owner != r) continue;
      if (hipMemcpy2DAsync(sbuf + off, b.r.w * sizeof(double), b.origin(s->cur), b.pitch * sizeof(double),
                           b.r.w * sizeof(double), b.r.h, hipMemcpyDeviceToDevice, s->s_comm) != hipSuccess)
        status = fail(NLH_ERR_HIP, "gather pack");
      off += b.r.w * b.r.h;
    }
  };
  std::vector<double> h;
  auto unpack = [&](int r) {
    h.resize(count[r]);
    if (hipMemcpyAsync(h.data(), rbuf, count[r] * sizeof(double), hipMemcpyDeviceToHost, s->s_comm) != hipSuccess ||
        hipStreamSynchronize(s->s_comm) != hipSuccess) {
      status = fail(NLH_ERR_HIP, "gather copy");
      return;
    }
    int64_t off = 0;
    for (auto &b : s->plan.blocks) {
      if (b.rank != r) continue;
      for (int64_t y = 0; y < b.r.h; ++y)
        std::memcpy(u + (b.r.y0 + y) * s->p.nx + b.r.x0, h.data() + off + y * b.r.w, b.r.w * sizeof(double));
      off += b.r.w * b.r.h;
    }
  };
  for (int r = 0; r < s->owners && status == NLH_OK; ++r) {
    if (r == root || !count[r]) continue;
    const bool sender = runs(s, r);
    if (!sender && !at_root) continue;
    if (sender) pack(r);
    if (status != NLH_OK) break;
    bool ok = ncclGroupStart() == ncclSuccess;
    const int to = s->vranks ? 0 : root, from = s->vranks ? 0 : r;
    if (sender) ok = ok && p2p(true, sbuf, count[r], to, s->comm, s->s_comm);
    if (at_root) ok = ok && p2p(false, rbuf, count[r], from, s->comm, s->s_comm);
    ok = (ncclGroupEnd() == ncclSuccess) && ok;
    if (!ok) {
      status = fail(NLH_ERR_RCCL, "gather send/recv");
      break;
    }
    if (at_root) unpack(r);
    if (hipStreamSynchronize(s->s_comm) != hipSuccess && status == NLH_OK) status = fail(NLH_ERR_HIP, "gather sync");
  }
  (void)hipFree(sbuf);
  (void)hipFree(rbuf);
  return status;
}

int nlh_barrier(nlh_solver *s) {
  if (!s) return fail(NLH_ERR_ARG, "null solver");
  int rc = set_device(s);
  if (rc) return rc;
  if (s->sync_mode != 0) {
    HIP_TRY(hipStreamSynchronize(s->s_main));
    HIP_TRY(hipStreamSynchronize(s->s_comm));
  } else if ((rc = poll_stream(s, s->s_main, false)) || (rc = poll_stream(s, s->s_comm, false))) {
    return rc;
  }
  if (s->comm) {
    NCCL_TRY(ncclAllReduce(s->d_red, s->d_red, 1, ncclDouble, ncclSum, s->comm, s->s_comm));
    HIP_TRY(hipStreamSynchronize(s->s_comm));
  }
  return NLH_OK;
}

int nlh_snapshot_begin(nlh_solver *s) {
  if (!s) return fail(NLH_ERR_ARG, "null solver");
  if (s->snap_pending) return fail(NLH_ERR_STATE, "a snapshot is already in flight (call nlh_snapshot_wait)");
  int rc = set_device(s);
  if (rc) return rc;
  int64_t owned = 0;
  for (auto &b : s->blocks) owned += b.r.w * b.r.h;
  if (!s->snap_dev) {  // first snapshot: buffers and the copy stream
    HIP_TRY(hipMalloc(&s->snap_dev, std::max<int64_t>(owned, 1) * sizeof(double)));
    HIP_TRY(hipHostMalloc(&s->snap_host, std::max<int64_t>(owned, 1) * sizeof(double), hipHostMallocDefault));
    HIP_TRY(hipStreamCreateWithFlags(&s->s_copy, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_snap_dev, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_snap, hipEventDisableTiming));
    s->device_bytes += owned * (int64_t)sizeof(double);
  }
  // the device copy sits on the step stream behind every enqueued pass (its
  // last bands included, nlh_run ends s_main on them), so the next pass cannot
  // overwrite the parity buffer before it is read; the slow host transfer then
  // runs on s_copy beside the following passes
  int64_t off = 0;
  for (auto &b : s->blocks) {
    HIP_TRY(hipMemcpy2DAsync(s->snap_dev + off, b.r.w * sizeof(double), b.origin(s->cur),
                             b.pitch * sizeof(double), b.r.w * sizeof(double), b.r.h,
                             hipMemcpyDeviceToDevice, s->s_main));
    off += b.r.w * b.r.h;
  }
  HIP_TRY(hipEventRecord(s->ev_snap_dev, s->s_main));
  HIP_TRY(hipStreamWaitEvent(s->s_copy, s->ev_snap_dev, 0));
  HIP_TRY(hipMemcpyAsync(s->snap_host, s->snap_dev, std::max<int64_t>(owned, 1) * sizeof(double),
                         hipMemcpyDeviceToHost, s->s_copy));
  HIP_TRY(hipEventRecord(s->ev_snap, s->s_copy));
  s->snap_pending = true;
  return NLH_OK;
}

int nlh_snapshot_wait(nlh_solver *s, double *u) {
  if (!s || !u) return fail(NLH_ERR_ARG, "null argument");
  if (!s->snap_pending) return fail(NLH_ERR_STATE, "no snapshot in flight");
  HIP_TRY(hipEventSynchronize(s->ev_snap));
  int64_t off = 0;
  for (auto &b : s->blocks) {
    for (int64_t y = 0; y < b.r.h; ++y)
      std::memcpy(u + (b.r.y0 + y) * s->p.nx + b.r.x0, s->snap_host + off + y * b.r.w, b.r.w * sizeof(double));
    off += b.r.w * b.r.h;
  }
  s->snap_pending = false;
  return NLH_OK;
}

int nlh_run(nlh_solver *s, int64_t nsteps) {
  if (!s) return fail(NLH_ERR_ARG, "null solver");
  if (nsteps < 0) return fail(NLH_ERR_ARG, "negative step count");
  s->h_enter = s->h_return = now_ns();  // h_return moves on only when the run was enqueued
  s->h_start_seen = s->h_end_seen = -1;
  s->h_sync_return = 0;
  s->h_e0 = s->h_e1 = nullptr;
  int rc = set_device(s);
  if (rc) return rc;
  if (nsteps == 0) return NLH_OK;
  if (s->timing != 0 && s->ev_used >= kEvFold && (rc = fold_events(s, false))) return rc;
  // timing 1 / 3: one event pair on the stencil stream around the whole call,
  // so back-to-back passes are not separated by per-launch event records
  TimedPair run_pair{s};
  const bool per_run = s->timing == 1 || s->timing == 3;
  if (per_run) {
    if ((rc = run_pair.begin(s->s_main, kEvRun))) return rc;
    s->h_e0 = s->ev_pool[s->ev_used - 2];
    s->h_e1 = run_pair.e1;
  }
  int64_t i = 0;
  // busy and phase timing record 2-4 event pairs per pass: fold the completed
  // ones every kEvFold events inside one long call too, so the pool stays
  // bounded
  auto fold = [&] { return s->timing >= 2 && s->ev_used >= kEvFold ? fold_events(s, false) : (int)NLH_OK; };
  // NLH_HOST_PROBE (diagnostics): after the first pass is enqueued, spin until
  // the run's start event has completed -- the host time the GPU took to
  // begin the run (the rest of the passes are enqueued while it runs)
  auto probe = [&] {
    if (!s->host_probe || !s->h_e0 || s->h_start_seen >= 0) return (int)NLH_OK;
    for (;;) {
      const hipError_t q = hipEventQuery(s->h_e0);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) return fail(NLH_ERR_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
    }
    s->h_start_seen = now_ns();
    return (int)NLH_OK;
  };
  const int spp = s->pair ? 2 : 1;
  while (i + spp <= nsteps) {
    if (const int g = graph_passes(s, (nsteps - i) / spp)) {
      if ((rc = launch_graph(s, g, spp)) || (rc = probe())) return rc;
      i += (int64_t)g * spp;
      continue;
    }
    if ((rc = enqueue_step(s, spp)) || (rc = fold()) || (rc = probe())) return rc;
    i += spp;
  }
  for (; i < nsteps; ++i)
    if ((rc = enqueue_step(s, 1)) || (rc = fold()) || (rc = probe())) return rc;
  if (s->exchange) HIP_TRY(hipStreamWaitEvent(s->s_main, s->ev_band, 0));  // last bands
  if (per_run && (rc = run_pair.end(s->s_main))) return rc;
  s->h_return = now_ns();
  return NLH_OK;
}

int nlh_synchronize(nlh_solver *s) {
  if (!s) return fail(NLH_ERR_ARG, "null solver");
  int rc = set_device(s);
  if (rc) return rc;
  if (s->sync_mode != 0) {
    HIP_TRY(hipStreamSynchronize(s->s_comm));
    HIP_TRY(hipStreamSynchronize(s->s_main));
  } else {
    if ((rc = poll_stream(s, s->s_comm, false)) || (rc = poll_stream(s, s->s_main, true))) return rc;
  }
  s->h_sync_return = now_ns();
  return NLH_OK;
}

int nlh_host_time(nlh_solver *s, nlh_host_times *out) {
  if (!s || !out) return fail(NLH_ERR_ARG, "null argument");
  std::memset(out, 0, sizeof(*out));
  const double e = (double)s->h_enter;
  out->enqueue_us = (s->h_return - e) / 1e3;
  out->sync_return_us = s->h_sync_return >= s->h_return ? (s->h_sync_return - e) / 1e3 : -1.0;
  out->start_seen_us = s->h_start_seen >= 0 ? (s->h_start_seen - e) / 1e3 : -1.0;
  out->end_seen_us = s->h_end_seen >= 0 ? (s->h_end_seen - e) / 1e3 : -1.0;
  out->event_span_us = -1.0;
  if (s->h_e0 && s->h_e1 && hipEventQuery(s->h_e1) == hipSuccess) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->h_e0, s->h_e1) == hipSuccess) out->event_span_us = ms * 1e3;
  }
  out->sync_mode = s->sync_mode;
  return NLH_OK;
}

int64_t nlh_step_index(const nlh_solver *s) { return s ? s->t : -1; }

int nlh_errors(nlh_solver *s, int64_t time, double *l2, double *linf) {
  if (!s || !l2 || !linf) return fail(NLH_ERR_ARG, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  const double save_st = s->sc.st2pi, save_ct = s->sc.ct;
  set_time(s, time);
  for (size_t i = 0; i < s->blocks.size(); ++i) {
    const auto &b = s->blocks[i];
    if (nlh::launch_norms(b.origin(s->cur), b.pitch, (int)b.r.w, (int)b.r.h, (int)b.r.x0,
                          (int)b.r.y0, s->sc, s->d_part + s->part_off[i], s->s_main))
      return fail(NLH_ERR_HIP, "norm launch");
  }
  s->sc.st2pi = save_st;
  s->sc.ct = save_ct;
  std::vector<nlh::NormPartial> h(std::max(s->part_total, 1));
  if (s->part_total)
    HIP_TRY(hipMemcpyAsync(h.data(), s->d_part, s->part_total * sizeof(nlh::NormPartial),
                           hipMemcpyDeviceToHost, s->s_main));
  HIP_TRY(hipStreamSynchronize(s->s_main));
  // each (virtual) rank's partial sums over its blocks in block order, then
  // across ranks: RCCL all-reduce between real ranks, rank order between the
  // virtual ranks of this process (the self-communicator's all-reduce below
  // is then the identity)
  std::vector<double> e2r(s->owners, 0.0), eir(s->owners, 0.0);
  for (size_t bi = 0; bi < s->blocks.size(); ++bi) {
    const int o = s->blocks[bi].owner;
    const int end = bi + 1 < s->blocks.size() ? s->part_off[bi + 1] : s->part_total;
    for (int i = s->part_off[bi]; i < end; ++i) {
      e2r[o] += h[i].l2;
      eir[o] = std::max(eir[o], h[i].linf);
    }
  }
  double e2 = 0.0, ei = 0.0;
  for (int r : s->mine) {
    e2 += e2r[r];
    ei = std::max(ei, eir[r]);
  }
  if (s->comm) {
    double v[2] = {e2, ei};
    HIP_TRY(hipMemcpyAsync(s->d_red, v, 2 * sizeof(double), hipMemcpyHostToDevice, s->s_comm));
    NCCL_TRY(ncclGroupStart());
    NCCL_TRY(ncclAllReduce(s->d_red, s->d_red, 1, ncclDouble, ncclSum, s->comm, s->s_comm));
    NCCL_TRY(ncclAllReduce(s->d_red + 1, s->d_red + 1, 1, ncclDouble, ncclMax, s->comm, s->s_comm));
    NCCL_TRY(ncclGroupEnd());
    HIP_TRY(hipMemcpyAsync(v, s->d_red, 2 * sizeof(double), hipMemcpyDeviceToHost, s->s_comm));
    HIP_TRY(hipStreamSynchronize(s->s_comm));
    e2 = v[0];
    ei = v[1];
  }
  *l2 = e2;
  *linf = ei;
  return NLH_OK;
}

int nlh_get_info(const nlh_solver *s, nlh_info *info) {
  if (!s || !info) return fail(NLH_ERR_ARG, "null argument");
  std::memset(info, 0, sizeof(*info));
  info->kernel = s->kernel;
  info->device = s->device;
  info->nblocks = (int32_t)s->blocks.size();
  info->npeers = (int32_t)s->peers.size();
  for (auto &b : s->blocks) info->owned_nodes += b.r.w * b.r.h;
  info->disk_points = s->disk;
  info->halo_bytes_sent = s->halo_bytes;
  info->device_bytes = s->device_bytes;
  info->halo_width = s->halo;
  info->steps_per_pass = s->pair ? 2 : 1;
  info->owners = s->owners;
  info->comm_nranks = s->comm_nranks;
  info->comm_rank = s->comm_rank;
  const char *pk = s->pair ? "k_pair_split"
                           : s->wide ? "k_wide"
                           : s->prefix ? (s->prefix_waves > 1 ? "k_prefix_rtw" : s->p.eps > 224 ? "k_prefix_rtc" : "k_prefix_rt")
                           : s->weighted ? "k_weighted"
                           : s->kernel == NLH_KERNEL_FAST ? "k_fast"
                           : nlh::exact_lds_ok((int)s->p.eps, s->p.test != 0) ? "k_exact_lds" : "k_exact";
  std::snprintf(info->pass_kernel, sizeof(info->pass_kernel), "%s", pk);
  std::snprintf(info->arch, sizeof(info->arch), "%s", s->arch);
  return NLH_OK;
}

int nlh_kernel_timing(nlh_solver *s, int enable) {
  if (!s) return fail(NLH_ERR_ARG, "null solver");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_main));
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  HIP_TRY(hipStreamSynchronize(s->s_band));
  s->timing = (enable == 2 || enable == 3) ? enable : enable != 0 ? 1 : 0;
  s->ev_used = 0;
  if (s->timing == 1 || s->timing == 3) {
    // the run pair's two events exist and have been recorded once before the
    // first timed nlh_run: creating and first recording them inside it
    // delayed its first launch (r06, tools/host_gap.py: the first timed runs
    // of a process start their passes 6-9 us later than the rest)
    while (s->ev_pool.size() < 2) {
      hipEvent_t e;
      HIP_TRY(hipEventCreate(&e));
      s->ev_pool.push_back(e);
    }
    HIP_TRY(hipEventRecord(s->ev_pool[0], s->s_main));
    HIP_TRY(hipEventRecord(s->ev_pool[1], s->s_main));
    HIP_TRY(hipStreamSynchronize(s->s_main));
  }
  s->ev_meta.clear();
  for (double &v : s->ev_acc_kind) v = 0.0;
  s->timed_steps = 0;
  s->timed_passes = 0;
  s->ev_acc_owner.assign(s->owners, 0.0);
  if (s->timing == 2) {
    // what a busy pair costs beyond its kernels' work: a pair
    // around ONE empty launch (t1) and around kK of them (tK), the least of a
    // few tries each; one more launch costs (tK - t1) / (kK - 1), the pair
    // itself t1 minus one launch -- fold_pair subtracts the pair's cost once
    // and the launch cost per launch it brackets
    constexpr int kTries = 8, kK = 8;
    for (int i = 0; i < 2 * kTries; ++i) {
      const hipEvent_t e0 = pool_event(s), e1 = pool_event(s);
      if (!e0 || !e1) return fail(NLH_ERR_HIP, "event pool");
      HIP_TRY(hipEventRecord(e0, s->s_main));
      for (int j = 0; j < (i < kTries ? 1 : kK); ++j)
        if (nlh::launch_noop(s->s_main)) return fail(NLH_ERR_HIP, "no-op launch");
      HIP_TRY(hipEventRecord(e1, s->s_main));
    }
    HIP_TRY(hipStreamSynchronize(s->s_main));
    float t1 = 0.f, tk = 0.f;
    for (int i = 0; i < 2 * kTries; ++i) {
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, s->ev_pool[2 * i], s->ev_pool[2 * i + 1]));
      float &best = i < kTries ? t1 : tk;
      best = (i == 0 || i == kTries) ? ms : std::min(best, ms);
    }
    const double per = std::max(0.0, (double)(tk - t1) / (kK - 1));
    s->launch_overhead_ms = per;
    s->pair_overhead_ms = std::max(0.0, (double)t1 - per);
    s->ev_used = 0;
  }
  return NLH_OK;
}

int nlh_kernel_time(nlh_solver *s, double *total_ms, int64_t *steps_out) {
  if (!s || !total_ms || !steps_out) return fail(NLH_ERR_ARG, "null argument");
  int rc = set_device(s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->s_main));
  HIP_TRY(hipStreamSynchronize(s->s_comm));
  HIP_TRY(hipStreamSynchronize(s->s_band));
  if ((rc = fold_events(s, true))) return rc;
  if (s->timing == 2) {
    double tot = 0.0;
    for (double v : s->ev_acc_kind) tot += v;
    *total_ms = tot;
  } else {
    *total_ms = s->ev_acc_kind[kEvRun];
  }
  *steps_out = s->timed_steps;
  return NLH_OK;
}

int nlh_phase_time(nlh_solver *s, nlh_phase_times *out) {
  if (!s || !out) return fail(NLH_ERR_ARG, "null argument");
  if (s->timing != 3) return fail(NLH_ERR_STATE, "phase timing is off (nlh_kernel_timing(s, 3))");
  int rc = set_device(s);
  if (rc) return rc;
  if ((rc = fold_events(s, true))) return rc;
  out->wall_ms = s->ev_acc_kind[kEvRun];
  out->interior_ms = s->ev_acc_kind[kEvInterior];
  out->band_ms = s->ev_acc_kind[kEvBand];
  out->exchange_ms = s->ev_acc_kind[kEvExchange];
  out->passes = s->timed_passes;
  out->steps = s->timed_steps;
  return NLH_OK;
}

int nlh_resolve_owner(int64_t tiles_x, int64_t tiles_y, int32_t nranks,
                      const int32_t *owner_in, int32_t *owner_out) {
  if (tiles_x < 1 || tiles_y < 1 || nranks < 1 || !owner_out) return fail(NLH_ERR_ARG, "bad argument");
  std::vector<int32_t> o;
  std::string err;
  if (!nlh::resolve_owner(tiles_x, tiles_y, nranks, owner_in, o, err)) return fail(NLH_ERR_ARG, err);
  std::memcpy(owner_out, o.data(), o.size() * sizeof(int32_t));
  return NLH_OK;
}

int64_t nlh_halo_plan(const nlh_params *p, int64_t *pieces, int64_t cap) {
  if (!p) return -fail(NLH_ERR_ARG, "null params");
  const int64_t tx = p->tiles_x > 0 ? p->tiles_x : 1, ty = p->tiles_y > 0 ? p->tiles_y : 1;
  if (p->nx <= 0 || p->ny <= 0 || p->nx % tx || p->ny % ty || p->nranks < 1)
    return -fail(NLH_ERR_ARG, "bad lattice / tile grid");
  std::vector<int32_t> o;
  std::string err;
  if (!nlh::resolve_owner(tx, ty, p->nranks, p->owner, o, err)) return -fail(NLH_ERR_ARG, err);
  // the halo width production resolves for these parameters (eps, or 2*eps
  // for the two-step pass)
  Resolved rv;
  if (int rc = resolve_config(*p, rv)) return -rc;
  nlh::Plan plan = nlh::make_plan(p->nx, p->ny, rv.halo, tx, ty, o, p->split_tiles == 0);
  int64_t n = 0;
  for (auto &pc : plan.pieces) {
    if (pc.dst_rank != p->rank) continue;
    if (pieces && n < cap) {
      int64_t *r = pieces + 8 * n;
      r[0] = pc.src_rank;
      r[1] = pc.dst_rank;
      r[2] = pc.r.x0;
      r[3] = pc.r.y0;
      r[4] = pc.r.w;
      r[5] = pc.r.h;
      r[6] = pc.src_block;
      r[7] = pc.dst_block;
    }
    ++n;
  }
  return n;
}

int64_t nlh_exchange_plan(const nlh_params *p, int64_t *out, int64_t cap) {
  if (!p) return -fail(NLH_ERR_ARG, "null params");
  const int64_t tx = p->tiles_x > 0 ? p->tiles_x : 1, ty = p->tiles_y > 0 ? p->tiles_y : 1;
  if (p->nx <= 0 || p->ny <= 0 || p->nx % tx || p->ny % ty || p->nranks < 1 || p->rank < 0 ||
      p->rank >= p->nranks)
    return -fail(NLH_ERR_ARG, "bad lattice / tile grid / rank");
  std::vector<int32_t> o;
  std::string err;
  if (!nlh::resolve_owner(tx, ty, p->nranks, p->owner, o, err)) return -fail(NLH_ERR_ARG, err);
  Resolved rv;
  if (int rc = resolve_config(*p, rv)) return -rc;
  nlh::Plan plan = nlh::make_plan(p->nx, p->ny, rv.halo, tx, ty, o, p->split_tiles == 0);
  const auto lay = nlh::exchange_layout(plan, p->rank, false);
  for (size_t i = 0; out && i < lay.size() && (int64_t)i < cap; ++i) {
    const auto &e = lay[i];
    const nlh::Piece &pc = plan.pieces[e.piece];
    int64_t *r = out + 8 * i;
    r[0] = e.peer;
    r[1] = e.dir;
    r[2] = e.offset;
    r[3] = pc.r.x0;
    r[4] = pc.r.y0;
    r[5] = pc.r.w;
    r[6] = pc.r.h;
    r[7] = e.piece;
  }
  return (int64_t)lay.size();
}

#ifndef NLH_BUILD_ID
#error "NLH_BUILD_ID must be defined by the build (Makefile: hash of the library sources)"
#endif
const char *nlh_build_id(void) { return NLH_BUILD_ID; }

int64_t nlh_block_plan(const nlh_params *p, int64_t *blocks, int64_t cap) {
  if (!p) return -fail(NLH_ERR_ARG, "null params");
  const int64_t tx = p->tiles_x > 0 ? p->tiles_x : 1, ty = p->tiles_y > 0 ? p->tiles_y : 1;
  if (p->nx <= 0 || p->ny <= 0 || p->nx % tx || p->ny % ty || p->nranks < 1)
    return -fail(NLH_ERR_ARG, "bad lattice / tile grid");
  std::vector<int32_t> o;
  std::string err;
  if (!nlh::resolve_owner(tx, ty, p->nranks, p->owner, o, err)) return -fail(NLH_ERR_ARG, err);
  // the halo width production resolves for these parameters (eps, or 2*eps
  // for the two-step pass)
  Resolved rv;
  if (int rc = resolve_config(*p, rv)) return -rc;
  nlh::Plan plan = nlh::make_plan(p->nx, p->ny, rv.halo, tx, ty, o, p->split_tiles == 0);
  int64_t n = 0;
  for (auto &b : plan.blocks) {
    if (blocks && n < cap) {
      int64_t *r = blocks + 6 * n;
      r[0] = b.rank;
      r[1] = b.local;
      r[2] = b.r.x0;
      r[3] = b.r.y0;
      r[4] = b.r.w;
      r[5] = b.r.h;
    }
    ++n;
  }
  return n;
}

int nlh_balance_owner(int64_t tiles_x, int64_t tiles_y, int32_t nranks, const int32_t *owner,
                      const double *busy, int32_t *owner_out) {
  if (tiles_x < 1 || tiles_y < 1 || nranks < 1 || !owner || !busy || !owner_out)
    return -fail(NLH_ERR_ARG, "bad argument");
  std::vector<int32_t> o, out;
  std::string err;
  if (!nlh::resolve_owner(tiles_x, tiles_y, nranks, owner, o, err)) return -fail(NLH_ERR_ARG, err);
  for (int r = 0; r < nranks; ++r)
    if (!(busy[r] >= 0.0)) return -fail(NLH_ERR_ARG, "busy times must be finite and >= 0");
  const int moved = nlh::balance_owner(tiles_x, tiles_y, nranks, o, busy, out);
  std::memcpy(owner_out, out.data(), out.size() * sizeof(int32_t));
  return moved;
}

int nlh_partition_tiles(int64_t tiles_x, int64_t tiles_y, int32_t nparts, const double *tile_weight,
                        int32_t *owner_out) {
  if (tiles_x < 1 || tiles_y < 1 || nparts < 1 || !owner_out) return fail(NLH_ERR_ARG, "bad argument");
  if (tile_weight)
    for (int64_t i = 0; i < tiles_x * tiles_y; ++i)
      if (!(tile_weight[i] >= 0.0)) return fail(NLH_ERR_ARG, "tile weights must be finite and >= 0");
  std::vector<int32_t> o;
  nlh::partition_tiles(tiles_x, tiles_y, nparts, tile_weight, o);
  std::memcpy(owner_out, o.data(), o.size() * sizeof(int32_t));
  return NLH_OK;
}

int nlh_repartition(nlh_solver *s, const int32_t *owner) {
  if (!s || !owner) return fail(NLH_ERR_ARG, "null argument");
  std::vector<int32_t> o;
  std::string err;
  if (!nlh::resolve_owner(s->p.tiles_x, s->p.tiles_y, s->owners, owner, o, err)) return fail(NLH_ERR_ARG, err);
  return repartition_impl(s, o);
}

int nlh_rebalance(nlh_solver *s, const double *busy_in, int32_t apply, int32_t *owner_out,
                  double *busy_out) {
  if (!s) return -fail(NLH_ERR_ARG, "null solver");
  int rc = set_device(s);
  if (rc) return -rc;
  const int R = s->owners;
  std::vector<double> busy(R, 0.0);
  if (busy_in) {
    for (int r = 0; r < R; ++r) busy[r] = busy_in[r];
  } else {
    if (s->timing != 2) return -fail(NLH_ERR_STATE, "busy timing is off (nlh_kernel_timing(s, 2))");
    std::vector<double> per;
    if ((rc = owner_busy(s, per))) return -rc;
    // virtual ranks: each one's own measured launch groups (their lists are
    // launched and timed separately); a real rank: its own, then all-gathered
    for (int r = 0; r < R; ++r) busy[r] = per[r];
    const double mine = per[s->p.rank];
    if (s->comm && R > 1 && R == s->p.nranks && !s->vranks) {
      double *d = nullptr;
      if (hipMalloc(&d, (R + 1) * sizeof(double)) != hipSuccess) return -fail(NLH_ERR_HIP, "busy buffer");
      int st = NLH_OK;
      if (hipMemcpyAsync(d + R, &mine, sizeof(double), hipMemcpyHostToDevice, s->s_comm) != hipSuccess)
        st = fail(NLH_ERR_HIP, "busy upload");
      if (st == NLH_OK && ncclAllGather(d + R, d, 1, ncclDouble, s->comm, s->s_comm) != ncclSuccess)
        st = fail(NLH_ERR_RCCL, "busy all-gather");
      if (st == NLH_OK && hipMemcpyAsync(busy.data(), d, R * sizeof(double), hipMemcpyDeviceToHost, s->s_comm) != hipSuccess)
        st = fail(NLH_ERR_HIP, "busy download");
      if (hipStreamSynchronize(s->s_comm) != hipSuccess && st == NLH_OK) st = fail(NLH_ERR_HIP, "busy sync");
      (void)hipFree(d);
      if (st) return -st;
    }
  }
  if (busy_out) std::memcpy(busy_out, busy.data(), R * sizeof(double));
  int moved = 0;
  if (apply) {
    for (int r = 0; r < R; ++r)
      if (!(busy[r] >= 0.0)) return -fail(NLH_ERR_ARG, "busy times must be finite and >= 0");
    std::vector<int32_t> next;
    moved = nlh::balance_owner(s->p.tiles_x, s->p.tiles_y, R, s->owner, busy.data(), next);
    if (moved > 0 && (rc = repartition_impl(s, next))) return -rc;
    if (s->timing == 2 && (rc = nlh_kernel_timing(s, 2))) return -rc;  // a new busy window
  }
  if (owner_out) std::memcpy(owner_out, s->owner.data(), s->owner.size() * sizeof(int32_t));
  return moved;
}

}  // extern "C"
