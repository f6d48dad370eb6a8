// 1d_nonlocal_serial -- drop-in for the reference executable of the same name
// (/root/reference/src/1d_nonlocal_serial.cpp), one MI355X through libnlh's
// nlh1d_* entry points.
//
// Same flags and defaults (:318-340), same stdin formats (batch :239-257:
// "num_tests" then rows "nx nt eps k dt dx"; IC :116-121, nx values), same
// stdout (banner, "l2: .. linfinity: ..", "Expected: .. Actual: ..",
// "S[x] = ..", "Tests Passed/Failed", the 1d timing line) and the same
// ../out_csv/{simulate,score}_1d.csv and ../out_vtk/simulate_<t/nlog> logs.
// Extra flag: --device N.
#include <sys/stat.h>

#include <cmath>
#include <cstdint>
#include <ctime>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "driver_common.h"
#include "nlh.h"
#include "vtu_writer.h"

using namespace nlh_drv;

namespace {

bool is_dir(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

struct Logger1d {
  int64_t nx = 0;
  double dt = 0, dx = 0;
  bool test = false, csv_ok = false, vtk_ok = false;
  void probe() {
    csv_ok = is_dir("../out_csv");
    vtk_ok = is_dir("../out_vtk");
  }
  bool enabled() const { return csv_ok || vtk_ok; }
  // log_vtk(t / nlog) and log_csv(t) of S[next] after step t (1d :132-167)
  void log(int64_t t, int64_t vtk_index, const std::vector<double> &u) const {
    if (vtk_ok) {
      VtuWriter v("../out_vtk/simulate_" + std::to_string(vtk_index));
      v.append_lattice_nodes(nx, 1);
      v.append_point_data("Temperature", u);
      v.add_time_step((double)std::time(nullptr));
      v.close();
    }
    if (!csv_ok) return;
    std::ofstream out("../out_csv/simulate_1d.csv", std::ios_base::app);
    double l2 = 0, linf = 0;
    const double ct = cos(2 * M_PI * (t * dt));
    for (int64_t x = 0; x < nx; ++x) {
      const double w = ct * sin(2 * M_PI * (x * dx)), d = u[x] - w;
      out << t << "," << x << "," << u[x] << "," << w << "," << d * d << "," << std::abs(d) << ",\n";
      l2 += d * d;
      linf = std::max(std::abs(d), linf);
    }
    if (test) {
      std::ofstream sc("../out_csv/score_1d.csv", std::ios_base::app);
      sc << t << "," << l2 << "," << linf << ",\n";
    }
  }
};

nlh1d_params make_params(int64_t nx, int64_t eps, double k, double dt, double dx, bool test, int device) {
  nlh1d_params p{};
  p.nx = nx;
  p.eps = eps;
  p.k = k;
  p.dt = dt;
  p.dx = dx;
  p.test = test;
  p.device = device;
  return p;
}

// do_work's loop (1d :209-236): steps between log points run back to back
int do_work(nlh1d_solver *s, int64_t nt, int64_t nlog, const Logger1d &lg) {
  std::vector<double> u(lg.nx);
  int64_t t = 0;
  while (t < nt) {
    int64_t stop = nt;  // the next step whose result is logged, inclusive
    if (lg.enabled() && nlog > 0) stop = std::min<int64_t>(nt, (t + nlog - 1) / nlog * nlog + 1);
    if (nlh1d_run(s, stop - t) != NLH_OK) return 1;
    t = stop;
    if (lg.enabled() && nlog > 0 && (t - 1) % nlog == 0) {
      if (nlh1d_get_field(s, u.data()) != NLH_OK) return 1;
      lg.log(t - 1, (t - 1) / nlog, u);
    }
  }
  return 0;
}

int batch_tester(int64_t nlog, int device) {
  uint64_t num_tests = 0;
  std::cin >> num_tests;
  bool failed = false;
  for (uint64_t i = 0; i < num_tests; ++i) {
    uint64_t nx, nt, eps;
    double k, dt, dx;
    std::cin >> nx >> nt >> eps >> k >> dt >> dx;
    nlh1d_params p = make_params(nx, eps, k, dt, dx, true, device);
    nlh1d_solver *s = nullptr;
    if (nlh1d_create(&p, &s) != NLH_OK) return die("nlh1d_create");
    if (nlh1d_init_test(s) != NLH_OK) return die("nlh1d_init_test");
    Logger1d lg;
    lg.nx = nx, lg.dt = dt, lg.dx = dx, lg.test = true;
    lg.probe();
    if (do_work(s, nt, nlog, lg)) return die("nlh1d_run");
    double l2 = 0, linf = 0;
    if (nlh1d_errors(s, nt, &l2, &linf) != NLH_OK) return die("nlh1d_errors");
    nlh1d_destroy(s);
    if (l2 / (double)nx > 1e-6) {
      failed = true;
      break;
    }
  }
  std::cout << (failed ? "Tests Failed" : "Tests Passed") << std::endl;
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  print_banner(argv[0]);
  Options o;
  o.flag("test");
  o.flag("test_batch");
  o.flag("results");
  o.opt("cmp", "true");
  o.opt("nx", "50");
  o.opt("nt", "45");
  o.opt("nlog", "5");
  o.opt("eps", "5");
  o.opt("k", "1");
  o.opt("dt", "0.001");
  o.opt("dx", "0.02");
  o.flag("no-header");
  o.opt("device", "-1");
  std::string err;
  if (!o.parse(argc, argv, err)) {
    std::cerr << err << std::endl;
    return 1;
  }
  const uint64_t nx = o.as_u64("nx"), nt = o.as_u64("nt"), eps = o.as_u64("eps"), nlog = o.as_u64("nlog");
  const double k = o.as_double("k"), dt = o.as_double("dt"), dx = o.as_double("dx");
  // the reference sets header = false for --no-header and never true (1d :27,277)
  const bool header = false;
  const int device = (int)o.as_i64("device");
  if (o.count("test_batch")) return batch_tester((int64_t)nlog, device);

  const bool test = o.count("test");
  nlh1d_params p = make_params(nx, eps, k, dt, dx, test, device);
  nlh1d_solver *s = nullptr;
  if (nlh1d_create(&p, &s) != NLH_OK) return die("nlh1d_create");
  if (test) {
    if (nlh1d_init_test(s) != NLH_OK) return die("nlh1d_init_test");
  } else {
    std::vector<double> u(nx, 0.0);
    for (auto &v : u) std::cin >> v;
    if (nlh1d_set_field(s, u.data()) != NLH_OK) return die("nlh1d_set_field");
  }
  Logger1d lg;
  lg.nx = nx, lg.dt = dt, lg.dx = dx, lg.test = test;
  lg.probe();
  const uint64_t t0 = now_ns();
  if (do_work(s, nt, nlog, lg)) return die("nlh1d_run");
  const uint64_t elapsed = now_ns() - t0;

  std::vector<double> u(nx);
  if (nlh1d_get_field(s, u.data()) != NLH_OK) return die("nlh1d_get_field");
  if (test) {
    double l2 = 0, linf = 0;
    if (nlh1d_errors(s, nt, &l2, &linf) != NLH_OK) return die("nlh1d_errors");
    print_errors(l2, linf);
    if (o.as_bool("cmp"))
      for (uint64_t x = 0; x < nx; ++x)
        std::cout << "Expected: " << cos(2 * M_PI * (nt * dt)) * sin(2 * M_PI * (x * dx)) << " Actual: " << u[x]
                  << std::endl;
  }
  if (o.count("results"))
    for (uint64_t x = 0; x < nx; ++x) std::cout << "S[" << x << "] = " << u[x] << std::endl;
  print_time_results(1, elapsed, nx, nt, header);
  nlh1d_destroy(s);
  return 0;
}
