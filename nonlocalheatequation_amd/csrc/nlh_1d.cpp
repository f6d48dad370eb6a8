// nlh_1d.cpp -- C ABI of the 1D solver (include/nlh.h, nlh1d_*): the
// drop-in for the reference's src/1d_nonlocal_serial.cpp.  Device field of
// nx + 2 eps doubles whose eps-wide frames stay 0 (the reference's
// boundary(), 1d :178-183); one launch of k_1d (nlh_kernels.hip) per step.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "nlh.h"

namespace nlh {
int launch_1d(const double *u, double *un, int64_t nx, int32_t eps, double c1d, double dt, double dx,
              bool test, double st2pi, double ct, const double *sxt, void *stream);
int launch_1d_norms(const double *u, int64_t nx, int32_t eps, double ct, const double *sxt, double *out,
                    void *stream);
const char *set_last_error(const std::string &msg);
}  // namespace nlh

struct nlh1d_solver {
  nlh1d_params p{};
  int device = 0;
  double c1d = 0;
  double *base[2] = {nullptr, nullptr};  // nx + 2 eps each, node x at base + eps + x
  double *d_sxt = nullptr;               // sin(2 pi (g dx)), g in [-eps, nx+eps)
  double *d_red = nullptr;               // {l2, linf}
  hipStream_t st = nullptr;
  int cur = 0;
  int64_t t = 0;
};

namespace {

int fail1d(int code, const std::string &msg) {
  nlh::set_last_error(msg);
  return code;
}

#define HIP1D(expr)                                                                           \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail1d(NLH_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

void destroy1d(nlh1d_solver *s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->st) (void)hipStreamSynchronize(s->st);
  (void)hipFree(s->base[0]);
  (void)hipFree(s->base[1]);
  (void)hipFree(s->d_sxt);
  (void)hipFree(s->d_red);
  if (s->st) (void)hipStreamDestroy(s->st);
  delete s;
}

int create1d(const nlh1d_params &p, nlh1d_solver *s) {
  if (p.nx <= 0) return fail1d(NLH_ERR_ARG, "nx must be positive");
  if (p.eps < 1) return fail1d(NLH_ERR_ARG, "eps must be >= 1");
  if (p.nx + 2 * p.eps > (1ll << 31)) return fail1d(NLH_ERR_ARG, "lattice too large");
  s->p = p;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail1d(NLH_ERR_HIP, "no HIP device visible (libnlh has no CPU fallback)");
  if (p.device >= ndev) return fail1d(NLH_ERR_ARG, "device ordinal out of range");
  if (p.device >= 0) s->device = p.device;
  else HIP1D(hipGetDevice(&s->device));
  HIP1D(hipSetDevice(s->device));
  hipDeviceProp_t prop;
  HIP1D(hipGetDeviceProperties(&prop, s->device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail1d(NLH_ERR_UNSUPPORTED, std::string("libnlh is built for gfx950, device is ") + prop.gcnArchName);
  // the reference's `long c_1d` (1d :57,74): truncated toward zero
  s->c1d = (double)(long)((p.k * 3) / (pow(p.eps * p.dx, 3)));
  const int64_t n = p.nx + 2 * p.eps;
  for (auto &b : s->base) {
    HIP1D(hipMalloc(&b, n * sizeof(double)));
    HIP1D(hipMemset(b, 0, n * sizeof(double)));
  }
  std::vector<double> sxt(n);
  for (int64_t g = -p.eps; g < p.nx + p.eps; ++g) sxt[g + p.eps] = sin(2 * M_PI * (g * p.dx));
  HIP1D(hipMalloc(&s->d_sxt, n * sizeof(double)));
  HIP1D(hipMemcpy(s->d_sxt, sxt.data(), n * sizeof(double), hipMemcpyHostToDevice));
  HIP1D(hipMalloc(&s->d_red, 2 * sizeof(double)));
  HIP1D(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
  return NLH_OK;
}

}  // namespace

extern "C" {

int nlh1d_create(const nlh1d_params *p, nlh1d_solver **out) {
  if (!p || !out) return fail1d(NLH_ERR_ARG, "null argument");
  *out = nullptr;
  nlh1d_solver *s = new nlh1d_solver();
  const int rc = create1d(*p, s);
  if (rc != NLH_OK) {
    const std::string keep = nlh_last_error();
    destroy1d(s);
    nlh::set_last_error(keep);
    return rc;
  }
  *out = s;
  return NLH_OK;
}

int nlh1d_destroy(nlh1d_solver *s) {
  destroy1d(s);
  return NLH_OK;
}

int nlh1d_init_test(nlh1d_solver *s) {
  if (!s) return fail1d(NLH_ERR_ARG, "null solver");
  HIP1D(hipSetDevice(s->device));
  // u(x, 0) = sin(2 pi (x dx)) = the table's interior (1d :124-129)
  HIP1D(hipMemcpyAsync(s->base[0] + s->p.eps, s->d_sxt + s->p.eps, s->p.nx * sizeof(double),
                       hipMemcpyDeviceToDevice, s->st));
  HIP1D(hipStreamSynchronize(s->st));
  s->cur = 0;
  s->t = 0;
  return NLH_OK;
}

int nlh1d_set_field(nlh1d_solver *s, const double *u) {
  if (!s || !u) return fail1d(NLH_ERR_ARG, "null argument");
  HIP1D(hipSetDevice(s->device));
  HIP1D(hipMemcpy(s->base[0] + s->p.eps, u, s->p.nx * sizeof(double), hipMemcpyHostToDevice));
  s->cur = 0;
  s->t = 0;
  return NLH_OK;
}

int nlh1d_get_field(nlh1d_solver *s, double *u) {
  if (!s || !u) return fail1d(NLH_ERR_ARG, "null argument");
  HIP1D(hipSetDevice(s->device));
  HIP1D(hipStreamSynchronize(s->st));
  HIP1D(hipMemcpy(u, s->base[s->cur] + s->p.eps, s->p.nx * sizeof(double), hipMemcpyDeviceToHost));
  return NLH_OK;
}

int nlh1d_run(nlh1d_solver *s, int64_t nsteps) {
  if (!s) return fail1d(NLH_ERR_ARG, "null solver");
  if (nsteps < 0) return fail1d(NLH_ERR_ARG, "negative step count");
  HIP1D(hipSetDevice(s->device));
  for (int64_t i = 0; i < nsteps; ++i) {
    // (2*M_PI)*(time*dt) as the reference spells it (1d :174, :187)
    const double arg = 2 * M_PI * (s->t * s->p.dt);
    const int rc = nlh::launch_1d(s->base[s->cur] + s->p.eps, s->base[1 - s->cur] + s->p.eps, s->p.nx,
                                  (int32_t)s->p.eps, s->c1d, s->p.dt, s->p.dx, s->p.test != 0,
                                  2 * M_PI * sin(arg), cos(arg), s->d_sxt, s->st);
    if (rc) return fail1d(NLH_ERR_HIP, std::string("1d step launch: ") + hipGetErrorString((hipError_t)rc));
    s->cur = 1 - s->cur;
    ++s->t;
  }
  HIP1D(hipStreamSynchronize(s->st));
  return NLH_OK;
}

int nlh1d_errors(nlh1d_solver *s, int64_t time, double *l2, double *linf) {
  if (!s || !l2 || !linf) return fail1d(NLH_ERR_ARG, "null argument");
  HIP1D(hipSetDevice(s->device));
  const double ct = cos(2 * M_PI * (time * s->p.dt));
  if (nlh::launch_1d_norms(s->base[s->cur] + s->p.eps, s->p.nx, (int32_t)s->p.eps, ct, s->d_sxt, s->d_red, s->st))
    return fail1d(NLH_ERR_HIP, "1d norm launch");
  double h[2];
  HIP1D(hipMemcpyAsync(h, s->d_red, sizeof(h), hipMemcpyDeviceToHost, s->st));
  HIP1D(hipStreamSynchronize(s->st));
  *l2 = h[0];
  *linf = h[1];
  return NLH_OK;
}

}  // extern "C"
