// 2d_nonlocal_serial -- drop-in for the reference executable of the same name
// (/root/reference/src/2d_nonlocal_serial.cpp), running the hot path on one
// MI355X through libnlh.
//
// Same flags and defaults (:387-411), same stdin formats (batch :306-333, IC
// :180-187 in x-outer order), same stdout (banner :383, "l2: .. linfinity:",
// "Expected: .. Actual: ..", "S[x][y] = ..", "Tests Passed/Failed", timing
// line :377) and the same ../out_csv, ../out_vtk logging.  Extra flags:
// --kernel auto|exact|fast, --device N.
#include <cstdint>
#include <iostream>
#include <string>
#include <vector>

#include "driver_common.h"
#include "nlh.h"

using namespace nlh_drv;

static int g_influence = NLH_INFLUENCE_CONSTANT;  // --influence (extra flag)

static nlh_params make_params(int64_t nx, int64_t ny, int64_t eps, double k, double dt, double dh,
                              bool test, int kernel, int device) {
  nlh_params p{};
  p.nx = nx;
  p.ny = ny;
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
  p.tiles_x = 1;
  p.tiles_y = 1;
  return p;
}

static int batch_tester(int64_t nlog, int kernel, int device) {
  uint64_t num_tests = 0;
  std::cin >> num_tests;
  bool failed = false;
  for (uint64_t i = 0; i < num_tests; ++i) {
    uint64_t nx, ny, nt, eps;
    double k, dt, dh;
    std::cin >> nx >> ny >> nt >> eps >> k >> dt >> dh;
    nlh_params p = make_params(nx, ny, eps, k, dt, dh, true, kernel, device);
    p.kernel = driver_kernel(p, (int64_t)nt);
    nlh_solver *s = nullptr;
    if (nlh_create(&p, &s) != NLH_OK) return die("nlh_create");
    note_fast_test_kernel(s, p, kernel, true);
    if (nlh_init_test(s) != NLH_OK) return die("nlh_init_test");
    Logger lg;
    lg.nx = nx, lg.ny = ny, lg.dt = dt, lg.dh = dh, lg.test = true;
    lg.probe();
    uint64_t el = 0;
    if (run_steps(s, nt, nlog, lg, false, 0, el) != NLH_OK) return die("nlh_run");
    double l2 = 0, linf = 0;
    if (nlh_errors(s, nt, &l2, &linf) != NLH_OK) return die("nlh_errors");
    nlh_destroy(s);
    if (l2 / (double)(nx * ny) > 1e-6) {
      failed = true;
      break;
    }
  }
  std::cout << (failed ? "Tests Failed" : "Tests Passed") << std::endl;
  return 0;
}

int main(int argc, char **argv) {
  print_banner(argv[0]);
  Options o;
  o.flag("test");
  o.flag("test_batch");
  o.flag("results");
  o.opt("cmp", "true");
  o.opt("nx", "50");
  o.opt("ny", "50");
  o.opt("nt", "45");
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
  const uint64_t nx = o.as_u64("nx"), ny = o.as_u64("ny"), nt = o.as_u64("nt");
  const uint64_t eps = o.as_u64("eps"), nlog = o.as_u64("nlog");
  const double k = o.as_double("k"), dt = o.as_double("dt"), dh = o.as_double("dh");
  const bool header = !o.count("no-header");
  const int kernel = kernel_from_name(o.str("kernel"));
  g_influence = influence_from_name(o.str("influence"));
  if (g_influence < 0) {
    std::cerr << "--influence must be constant or linear" << std::endl;
    return 1;
  }
  const int device = (int)o.as_i64("device");

  if (o.count("test_batch")) return batch_tester((int64_t)nlog, kernel, device);

  const bool test = o.count("test");
  nlh_params p = make_params(nx, ny, eps, k, dt, dh, test, kernel, device);
  p.kernel = driver_kernel(p, (int64_t)nt);
  nlh_solver *s = nullptr;
  if (nlh_create(&p, &s) != NLH_OK) return die("nlh_create");
  note_fast_test_kernel(s, p, kernel, true);
  if (test) {
    if (nlh_init_test(s) != NLH_OK) return die("nlh_init_test");
  } else {  // input_init: nx*ny values, sx outer (:180-187)
    std::vector<double> u(nx * ny, 0.0);
    for (uint64_t sx = 0; sx < nx; ++sx)
      for (uint64_t sy = 0; sy < ny; ++sy) std::cin >> u[sx + sy * nx];
    if (nlh_set_field(s, u.data()) != NLH_OK) return die("nlh_set_field");
  }

  Logger lg;
  lg.nx = nx, lg.ny = ny, lg.dt = dt, lg.dh = dh, lg.test = test;
  lg.probe();
  uint64_t elapsed = 0;
  if (run_steps(s, nt, nlog, lg, false, 0, elapsed) != NLH_OK) return die("nlh_run");

  std::vector<double> u;
  if (test || o.count("results")) {
    u.assign(nx * ny, 0.0);
    if (nlh_get_field(s, u.data()) != NLH_OK) return die("nlh_get_field");
  }
  if (test) {
    double l2 = 0, linf = 0;
    if (nlh_errors(s, nt, &l2, &linf) != NLH_OK) return die("nlh_errors");
    print_errors(l2, linf);
    if (o.as_bool("cmp"))
      for (uint64_t sx = 0; sx < nx; ++sx)
        for (uint64_t sy = 0; sy < ny; ++sy)
          std::cout << "Expected: " << w_exact(sx, sy, nt, dt, dh) << " Actual: " << u[sx + sy * nx]
                    << std::endl;
  }
  if (o.count("results")) {
    for (uint64_t sx = 0; sx < nx; ++sx) {
      for (uint64_t sy = 0; sy < ny; ++sy)
        std::cout << "S[" << sx << "][" << sy << "] = " << u[sx + sy * nx] << " ";
      std::cout << std::endl;
    }
  }
  print_time_results(1, elapsed, nx, ny, nt, header);
  nlh_destroy(s);
  return 0;
}
