// 2d_nonlocal_async -- drop-in for the reference executable of the same name
// (/root/reference/src/2d_nonlocal_async.cpp) on one MI355X through libnlh.
//
// The reference splits an (nx*np) x (ny*np) lattice into np x np tiles and
// runs one HPX dataflow task per tile per step, with the dependency depth
// bounded by --nd (:408-473).  Here the whole lattice is one device block and
// one kernel launch per step covers every tile; --np keeps its meaning for
// the lattice size and the output, --nd is accepted (launches are already
// queued asynchronously, so there is no dependency tree to throttle).
// Flags/defaults (:545-578), batch format (:478-504), outputs (:191-284, :540)
// as the reference; extra flags --kernel auto|exact|fast, --device N.
#include <cstdint>
#include <iostream>
#include <string>
#include <vector>

#include "driver_common.h"
#include "nlh.h"

using namespace nlh_drv;

static int g_influence = NLH_INFLUENCE_CONSTANT;  // --influence (extra flag)

static int solve(int64_t nx, int64_t ny, int64_t np, int64_t nt, int64_t eps, double k, double dt,
                 double dh, bool test, int64_t nlog, int kernel, int device, nlh_solver **out,
                 uint64_t &elapsed) {
  nlh_params p{};
  p.nx = nx * np;
  p.ny = ny * np;
  p.eps = eps;
  p.k = k;
  p.dt = dt;
  p.dh = dh;
  p.test = test;
  p.kernel = kernel;
  p.influence = g_influence;
  p.device = device;
  p.rank = 0;
  p.nranks = 1;
  p.tiles_x = np;
  p.tiles_y = np;
  p.kernel = driver_kernel(p, nt);
  if (nlh_create(&p, out) != NLH_OK) return die("nlh_create");
  note_fast_test_kernel(*out, p, kernel, true);
  // the partition_space constructor always applies the sin*sin IC (:70-78)
  if (nlh_init_test(*out) != NLH_OK) return die("nlh_init_test");
  Logger lg;
  lg.nx = p.nx, lg.ny = p.ny, lg.dt = dt, lg.dh = dh, lg.test = test;
  lg.probe();
  if (run_steps(*out, nt, nlog, lg, true, 0, elapsed) != NLH_OK) return die("nlh_run");
  return 0;
}

int main(int argc, char **argv) {
  print_banner(argv[0]);
  Options o;
  o.opt("test", "true");
  o.flag("test_batch");
  o.flag("results");
  o.opt("cmp", "false");
  o.opt("nx", "25");
  o.opt("ny", "25");
  o.opt("nt", "45");
  o.opt("nd", "5");
  o.opt("np", "2");
  o.opt("nlog", "5");
  o.opt("eps", "5");
  o.opt("k", "1");
  o.opt("dt", "0.0005");
  o.opt("dh", "0.02");
  o.flag("no-header");
  o.opt("kernel", "auto");
  o.opt("influence", "constant");
  o.opt("device", "-1");
  std::string err;
  if (!o.parse(argc, argv, err)) {
    std::cerr << err << std::endl;
    return 1;
  }
  const bool header = !o.count("no-header");
  const int kernel = kernel_from_name(o.str("kernel"));
  g_influence = influence_from_name(o.str("influence"));
  if (g_influence < 0) {
    std::cerr << "--influence must be constant or linear" << std::endl;
    return 1;
  }
  const int device = (int)o.as_i64("device");
  const int64_t nlog = (int64_t)o.as_u64("nlog");

  if (o.count("test_batch")) {
    uint64_t num = 0;
    std::cin >> num;
    bool failed = false;
    for (uint64_t i = 0; i < num; ++i) {
      int64_t nx, ny, np, nt, eps;
      double k, dt, dh;
      std::cin >> nx >> ny >> np >> nt >> eps >> k >> dt >> dh;
      nlh_solver *s = nullptr;
      uint64_t el = 0;
      if (solve(nx, ny, np, nt, eps, k, dt, dh, true, nlog, kernel, device, &s, el)) return 1;
      double l2 = 0, linf = 0;
      if (nlh_errors(s, nt, &l2, &linf) != NLH_OK) return die("nlh_errors");
      nlh_destroy(s);
      if (l2 / (double)(nx * ny * np * np) > 1e-6) {
        failed = true;
        break;
      }
    }
    std::cout << (failed ? "Tests Failed" : "Tests Passed") << std::endl;
    return 0;
  }

  const int64_t nx = o.as_i64("nx"), ny = o.as_i64("ny"), np = o.as_i64("np");
  const int64_t nt = (int64_t)o.as_u64("nt"), eps = o.as_i64("eps");
  const double k = o.as_double("k"), dt = o.as_double("dt"), dh = o.as_double("dh");
  const bool test = o.as_bool("test");
  nlh_solver *s = nullptr;
  uint64_t elapsed = 0;
  if (solve(nx, ny, np, nt, eps, k, dt, dh, test, nlog, kernel, device, &s, elapsed)) return 1;

  const int64_t gx = nx * np, gy = ny * np;
  std::vector<double> u;
  if (test || o.count("results")) {
    u.assign(gx * gy, 0.0);
    if (nlh_get_field(s, u.data()) != NLH_OK) return die("nlh_get_field");
  }
  if (test) {
    double l2 = 0, linf = 0;
    if (nlh_errors(s, nt, &l2, &linf) != NLH_OK) return die("nlh_errors");
    print_errors(l2, linf);
    if (o.as_bool("cmp"))
      for (int64_t sx = 0; sx < gx; ++sx)
        for (int64_t sy = 0; sy < gy; ++sy)
          std::cout << "Expected: " << w_exact(sx, sy, nt, dt, dh) << " Actual: " << u[sx + sy * gx]
                    << std::endl;
  }
  if (o.count("results")) {
    for (int64_t sx = 0; sx < gx; ++sx) {
      for (int64_t sy = 0; sy < gy; ++sy)
        std::cout << "S[" << sx << "][" << sy << "] = " << u[sx + sy * gx] << " ";
      std::cout << std::endl;
    }
  }
  print_time_results(1, elapsed, nx, ny, nt, header);
  nlh_destroy(s);
  return 0;
}
