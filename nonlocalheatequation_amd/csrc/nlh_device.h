// nlh_device.h -- structures shared by the host orchestration (nlh_api.cpp)
// and the gfx950 kernels (nlh_kernels.hip), plus the internal launch API.
//
// HBM layout of one block (a rectangle of owned nodes, bx x by):
//   padded rows  y in [-E, by+E)        E = eps
//   padded cols  x in [-XL, pitch-XL)   XL = round_up(eps, 8)
//   node (x, y) at  base + (y + E) * pitch + (x + XL)
// Everything outside the owned rectangle is a halo: zero where it lies
// outside the global domain (the reference's boundary() volume constraint,
// src/2d_nonlocal_serial.cpp:213-221), filled from neighbouring blocks each
// step otherwise.  The kernels therefore never test for the boundary.
#pragma once
#include <cstdint>

namespace nlh {

constexpr int kMaxRects = 32;
constexpr int kMaxCopies = 64;

// One output rectangle of a launch, in block-local node coordinates.
struct Rect {
  const double *u;    // node (0,0) of the current field
  double *un;         // node (0,0) of the next field
  const double *lw;   // node (0,0) of L_h[W0] (fast test mode) or nullptr
  int64_t pitch;      // doubles per padded row
  int32_t gx0, gy0;   // global coordinates of node (0,0)
  int32_t x0, y0, x1, y1;
  int32_t wg_begin;   // first work item of this rect
  int32_t nstrip;     // fast kernels: strips of output columns
  int32_t nseg;       // fast kernels: segments of seg_rows rows
  int32_t seg_rows;   // fast kernels: segment height of this rect
};

struct RectList {
  Rect r[kMaxRects];
  int32_t nrects;
  int32_t nwork;
  int32_t owner;  // host bookkeeping: the (virtual) rank owning every rect of the list
  int32_t pad_;
};

// Per-step constants.  All trig values are computed on the host with glibc
// so that w() is bit-identical to the reference's.
struct StepConst {
  double c2d;      // (k*8)/pow(eps*dh,4)           reference :76
  double dh2;      // dh*dh
  double dt;
  double alpha;    // c2d*dh2*dt            (fast kernel)
  double nf;       // N(eps) as double      (fast kernel)
  double st2pi;    // (2*pi)*sin(2*pi*(t*dt))
  double ct;       // cos(2*pi*(t*dt))
  const double *sxt;  // sin(2*pi*(g*dh)), g in [-E, nx+E), index g+E
  const double *syt;  // same over y
  const int32_t *lens;  // len_1d_line(|d|) for d in [0, E]
  int64_t nx, ny;  // global lattice
  int32_t E;
  int32_t seg_h;   // fast kernel segment height
  double kc;       // 1/alpha - N  (centre fold: pair and wide kernels)
  int32_t seg_pair;  // pair kernel segment height
  int32_t influence;  // nlh_influence: 0 = J = 1, else J from the tables below
  // J != 1: wt[n] = J*c2d per disk point in the reference's loop order (sx
  // outer, sy inner; k_exact), qj[dx*(E+1)+dy] = J(dx, dy) for the quadrant
  // 0 <= dy <= len(dx) (k_weighted), jsum = sum of J over the disk
  const double *wt;
  const double *qj;
  double jsum;
  double st2pi2;   // st2pi, ct at time t+1 (two-step test mode: the second step's source)
  double ct2;
  // separable L_h[W0] (two-step test mode, nlh_pair.h OPT & 32768):
  // L_h[W0](x, y) = sum_l Sx'_l(x) Ty_l(y) + sx(x) Z(y), c dh^2 folded into
  // lsx; lsx rows l < NLV: Sx'_l, row NLV: sx (0 outside the lattice), over
  // global columns -2E .. (stride pair_sep_ncol); lty rows y = -2E ..
  // ny+2E-1 (stride pair_sep_stride(E)): Ty_l(y) for l < NLV, Z(y) at NLV
  // (nlh_api.cpp sep_tables)
  const double *lsx;
  const double *lty;
};

// Strided rectangle copy (halo exchange: local block->block copies, pack to
// and unpack from RCCL message buffers).
struct Copy {
  const double *src;
  double *dst;
  int64_t spitch, dpitch;  // elements
  int32_t w, h;
  int32_t wg_begin;
  int32_t pad_;
};
struct CopyList {
  Copy c[kMaxCopies];
  int32_t ncopies;
  int32_t nwork;
};

struct NormPartial {
  double l2;
  double linf;
};

// ---- launch API (nlh_kernels.hip) -----------------------------------------
// Returns false if (E, R) has no fast instantiation.
bool fast_supported(int E);
int fast_lanes_cols(int E, int want_r);   // R actually used (2 or 4)
int fast_strip_width(int E, int want_r);  // 64*R columns per strip
int fast_seg_min(int E);                  // smallest sensible segment height
// Work-item counts are filled into rl by the caller (wg_begin/nwork).
int launch_fast(const RectList &rl, const StepConst &c, bool test, int want_r, void *stream);
// large horizons (nlh_wide.h, eps in [17, 48]): single-step, 64-column strips,
// centre fold (needs kc), production and fast test mode
bool wide_supported(int E);
int wide_blocks_per_cu(int E);  // resident k_wide workgroups per CU
int launch_wide(const RectList &rl, const StepConst &c, bool test, void *stream);
// two-step pass (nlh_pair.h): production mode, eps in [1, 16]
bool pair_supported(int E);
int pair_strip_width(int E);  // output columns per strip: 128 - 2E
// variant: k_pair_split's ring configuration (nlh_pair.h: 1 / 6 production,
// 5 / 4 test mode); all bitwise equal
int pair_blocks_per_cu(int E, int variant);  // resident workgroups per CU (0 = unknown)
// or'ed into variant 5 / 6: the same kernel without the wave priority (nlh_pair.h)
constexpr int kPairNoPrio = 0x100;

// separable L_h[W0] tables (StepConst lsx / lty; nlh_pair.h OPT & 32768):
// columns of lsx -- global -2E .. nx + 2E + 127 (a last strip's stage-1
// columns reach past the lattice; 0 there) -- and the lty row stride for nlv
// levels (nlv values + Z, a power of two)
constexpr int64_t pair_sep_ncol(int E, int64_t nx) { return nx + 4 * E + 128; }
constexpr int pair_sep_stride_n(int nlv) {
  int s = 1;
  while (s < nlv + 1) s *= 2;
  return s;
}
int launch_pair(const RectList &rl, const StepConst &c, int variant, void *stream);
int launch_exact(const RectList &rl, const StepConst &c, bool test, void *stream);
// fast path for a non-constant J (influence != 0, eps <= 32): LDS tile of
// 64 x 16 outputs per workgroup, direct weighted sum over the disk's 4-fold
// symmetric groups; rect lists as k_exact with 16-row segments
bool weighted_supported(int E);
// k_exact_lds (LDS-staged bit-parity kernel, 16-row segments) handles (E, test);
// otherwise k_exact (4-row segments)
bool exact_lds_ok(int E, bool test);
int launch_weighted(const RectList &rl, const StepConst &c, bool test, void *stream);
// A = sum_local(u) only (no time update) -- used once for L_h[W0].
int launch_exact_sum(const RectList &rl, const StepConst &c, void *stream);
int launch_copies(const CopyList &cl, void *stream);
int launch_noop(void *stream);  // one empty workgroup (launch-overhead probe)
// u(x,y) = sxt[gx]*syt[gy] on the block interior; halo untouched.
int launch_init_test(double *u, int64_t pitch, int32_t bx, int32_t by,
                     int32_t gx0, int32_t gy0, const StepConst &c, void *stream);
// W0 over the padded block INCLUDING its `halo` rows: sxt*syt inside the
// domain, 0 out.
int launch_fill_w0(double *u, int64_t pitch, int32_t xl, int32_t bx,
                   int32_t by, int32_t halo, int32_t gx0, int32_t gy0, const StepConst &c,
                   void *stream);
// L_h[W0] (fast test mode, J = 1) from the separable tables StepConst lsx /
// lty (nlv levels, lty row stride lts) over block-relative x0 .. x0+w,
// y0 .. y0+h of the plane whose node (0,0) is `out`; 0 outside the lattice.
int launch_lw_sep(double *out, int64_t pitch, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t gx0,
                  int32_t gy0, const StepConst &c, int32_t nlv, int32_t lts, void *stream);
// Partial L2/Linf per workgroup into `out` (nwg entries); returns nwg.
int norm_workgroups(int32_t bx, int32_t by);
int launch_norms(const double *u, int64_t pitch, int32_t bx, int32_t by,
                 int32_t gx0, int32_t gy0, const StepConst &c,
                 NormPartial *out, void *stream);

}  // namespace nlh
