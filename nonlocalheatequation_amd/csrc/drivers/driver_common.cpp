// driver_common.cpp -- see driver_common.h.
#include "driver_common.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <functional>
#include <iostream>
#include <thread>

#include "vtu_writer.h"

namespace nlh_drv {

// ---------------------------------------------------------------- options
void Options::flag(const std::string &name) { flags_[name] = false; }

void Options::opt(const std::string &name, const std::string &def) { vals_[name] = def; }

bool Options::parse(int argc, char **argv, std::string &err) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.rfind("--hpx:", 0) == 0) {  // HPX runtime options: accepted, ignored
      if (a.find('=') == std::string::npos && i + 1 < argc && argv[i + 1][0] != '-') ++i;
      continue;
    }
    if (a.rfind("--", 0) != 0) {
      err = "unexpected argument '" + a + "'";
      return false;
    }
    std::string name = a.substr(2), val;
    bool has_val = false;
    const size_t eq = name.find('=');
    if (eq != std::string::npos) {
      val = name.substr(eq + 1);
      name = name.substr(0, eq);
      has_val = true;
    }
    if (flags_.count(name)) {
      flags_[name] = true;
      continue;
    }
    if (!vals_.count(name)) {
      err = "unrecognised option '--" + name + "'";
      return false;
    }
    if (!has_val) {
      if (i + 1 >= argc) {
        err = "the required argument for option '--" + name + "' is missing";
        return false;
      }
      val = argv[++i];
    }
    vals_[name] = val;
  }
  return true;
}

bool Options::count(const std::string &name) const {
  auto it = flags_.find(name);
  return it != flags_.end() && it->second;
}

std::string Options::str(const std::string &name) const { return vals_.at(name); }

bool Options::as_bool(const std::string &name) const {
  std::string v = vals_.at(name);
  std::transform(v.begin(), v.end(), v.begin(), ::tolower);
  return v == "1" || v == "true" || v == "yes" || v == "on";
}

int64_t Options::as_i64(const std::string &name) const { return std::stoll(vals_.at(name)); }

uint64_t Options::as_u64(const std::string &name) const { return std::stoull(vals_.at(name)); }

double Options::as_double(const std::string &name) const { return std::stod(vals_.at(name)); }

// ---------------------------------------------------------------- output
// Every driver links this file: at start, before main, the libnlh the binary
// loaded must carry the build id the driver was compiled with (Makefile
// BUILD_ID over the library AND driver sources) -- a stale bin/ driver, or a
// library rebuilt without relinking the drivers, fails loudly instead of
// running an old code path.
#ifndef NLH_DRIVER_BUILD_ID
#error "compile driver_common.cpp with -DNLH_DRIVER_BUILD_ID (Makefile)"
#endif
namespace {
struct BuildIdCheck {
  BuildIdCheck() {
    const char *lib = nlh_build_id();
    if (!lib || std::strcmp(lib, NLH_DRIVER_BUILD_ID) != 0) {
      std::fprintf(stderr, "driver built for libnlh %s but loaded libnlh %s: rebuild with `make drivers`\n",
                   NLH_DRIVER_BUILD_ID, lib ? lib : "(none)");
      std::exit(3);
    }
  }
} g_build_id_check;
}  // namespace

void print_banner(const char *argv0) {
  // MAJOR.MINOR.UPDATE of include/Config.h (0.1.0)
  std::cout << argv0 << " (0.1.0)" << std::endl;
}

void print_time_results(uint64_t threads, uint64_t elapsed_ns, uint64_t nx, uint64_t ny,
                        uint64_t nt, bool header) {
  if (header)
    std::cout << "OS_Threads,       Execution_Time_sec,"
                 "       x dimension,        y dimension,        Time_Steps\n"
              << std::flush;
  const std::string t = std::to_string(threads) + ",", x = std::to_string(nx) + ",",
                    y = std::to_string(ny) + ",", n = std::to_string(nt) + " ";
  std::printf("%-21s %10.12lf,        %-21s %-21s %-21s\n", t.c_str(), elapsed_ns / 1e9, x.c_str(),
              y.c_str(), n.c_str());
  std::fflush(stdout);
}

void print_time_results(uint32_t localities, uint64_t threads, uint64_t elapsed_ns, uint64_t nx,
                        uint64_t ny, uint64_t npx, uint64_t npy, uint64_t nt, bool header) {
  if (header)
    std::cout << "Localities,OS_Threads,Execution_Time_sec,"
                 "       nx,    ny,     npx,    npy,    Time_Steps\n"
              << std::flush;
  const std::string l = std::to_string(localities) + ",", t = std::to_string(threads) + ",",
                    x = std::to_string(nx) + ",", y = std::to_string(ny) + ",",
                    px = std::to_string(npx) + ",", py = std::to_string(npy) + ",",
                    n = std::to_string(nt) + " ";
  std::printf("%-6s %-6s %.14g, %-21s %-21s %-21s %-21s %-21s\n", l.c_str(), t.c_str(),
              elapsed_ns / 1e9, x.c_str(), y.c_str(), px.c_str(), py.c_str(), n.c_str());
  std::fflush(stdout);
}

void print_time_results(uint64_t threads, uint64_t elapsed_ns, uint64_t nx, uint64_t nt, bool header) {
  if (header)
    std::cout << "OS_Threads,       Execution_Time_sec,"
                 "       x dimension,        y dimension,        Time_Steps\n"
              << std::flush;
  const std::string t = std::to_string(threads) + ",", x = std::to_string(nx) + ",",
                    n = std::to_string(nt) + " ";
  std::printf("%-21s %10.12lf,        %-21s %-21s\n", t.c_str(), elapsed_ns / 1e9, x.c_str(), n.c_str());
  std::fflush(stdout);
}

void print_errors(double l2, double linf) {
  std::cout << "l2: " << l2 << " linfinity: " << linf << std::endl;
}

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ---------------------------------------------------------------- ranks
static int env_int(const char *a, int def) {
  const char *v = std::getenv(a);
  return v ? std::atoi(v) : def;
}

RankEnv rank_env() {
  RankEnv r;
  const char *sets[][3] = {{"RANK", "WORLD_SIZE", "LOCAL_RANK"},
                           {"OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"},
                           {"SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"},
                           {"PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"}};
  for (auto &s : sets) {
    if (std::getenv(s[0]) && std::getenv(s[1])) {
      r.rank = env_int(s[0], 0);
      r.nranks = env_int(s[1], 1);
      r.local_rank = env_int(s[2], r.rank);
      break;
    }
  }
  return r;
}

static bool send_all(int fd, const void *p, size_t n) {
  const char *c = (const char *)p;
  while (n) {
    const ssize_t k = ::send(fd, c, n, 0);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

static bool recv_all(int fd, void *p, size_t n) {
  char *c = (char *)p;
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool share_comm_id(const RankEnv &re, uint8_t id[NLH_COMM_ID_BYTES], std::string &err, bool fresh) {
  const char *addr = std::getenv("MASTER_ADDR");
  const int port = env_int("MASTER_PORT", 29517) + 1;  // next to torch's own store port
  if (!addr) addr = "127.0.0.1";
  // every call is one bootstrap round (a batch row); a client names the
  // round it wants, and rank 0 serves only clients of its current round, so a
  // fast rank already at row r+1 cannot take row r's id
  static uint32_t round = 0;
  const uint32_t my_round = round++;
  if (re.rank == 0) {
    if (fresh && nlh_comm_unique_id(id) != NLH_OK) {
      err = nlh_last_error();
      return false;
    }
    const int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(lfd, (sockaddr *)&sa, sizeof(sa)) != 0 || ::listen(lfd, re.nranks) != 0) {
      err = "cannot listen on port " + std::to_string(port);
      ::close(lfd);
      return false;
    }
    for (int served = 1; served < re.nranks;) {
      const int fd = ::accept(lfd, nullptr, nullptr);
      if (fd < 0) {
        err = "bootstrap accept failed";
        ::close(lfd);
        return false;
      }
      uint32_t want = 0;
      // a client of another round is turned away (it retries)
      if (recv_all(fd, &want, sizeof(want)) && want == my_round && send_all(fd, id, NLH_COMM_ID_BYTES)) ++served;
      ::close(fd);
    }
    ::close(lfd);
    return true;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(addr, std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    err = std::string("cannot resolve MASTER_ADDR ") + addr;
    return false;
  }
  bool ok = false;
  for (int attempt = 0; attempt < 1200 && !ok; ++attempt) {  // up to ~60 s
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0)
      ok = send_all(fd, &my_round, sizeof(my_round)) && recv_all(fd, id, NLH_COMM_ID_BYTES);
    ::close(fd);
    if (!ok) std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  ::freeaddrinfo(res);
  if (!ok) err = "bootstrap: could not fetch the RCCL id from rank 0";
  return ok;
}

int influence_from_name(const std::string &s) {
  if (s == "constant") return NLH_INFLUENCE_CONSTANT;
  if (s == "linear") return NLH_INFLUENCE_LINEAR;
  return -1;
}

int kernel_from_name(const std::string &s) {
  if (s == "exact") return NLH_KERNEL_EXACT;
  if (s == "fast") return NLH_KERNEL_FAST;
  return NLH_KERNEL_AUTO;
}

int driver_kernel(const nlh_params &p, int64_t nt) {
  if (p.kernel != NLH_KERNEL_AUTO || !p.test) return p.kernel;
  int64_t n = 0;  // N(eps): the reference's disk count (len_1d_line, :231)
  for (int64_t dx = -p.eps; dx <= p.eps; ++dx) n += 2 * (int64_t)std::sqrt((double)(p.eps * p.eps - dx * dx)) + 1;
  const double terms = (double)p.nx * (double)p.ny * (double)std::max<int64_t>(nt, 1) * (double)n;
  return terms <= kDriverExactTerms ? NLH_KERNEL_EXACT : NLH_KERNEL_AUTO;
}

void note_fast_test_kernel(nlh_solver *s, const nlh_params &p, int requested, bool print) {
  if (!print || !p.test || requested != NLH_KERNEL_AUTO) return;
  nlh_info info{};
  if (nlh_get_info(s, &info) != NLH_OK || info.kernel != NLH_KERNEL_FAST) return;
  std::cerr << "note: --kernel auto ran the FAST kernel " << info.pass_kernel
            << " (test mode): every node within 1e-12 of the field scale of the reference's order, so l2 / "
               "linfinity match the reference's to 1e-10 relative where its error is above the rounding floor "
               "those node differences set, and within that bound below it (include/nlh.h); --kernel exact "
               "reproduces the reference's order bit for bit"
            << std::endl;
}

double w_exact(int64_t x, int64_t y, int64_t t, double dt, double dh) {
  return cos(2 * M_PI * (t * dt)) * sin(2 * M_PI * (x * dh)) * sin(2 * M_PI * (y * dh));
}

// ---------------------------------------------------------------- logging
static bool is_dir(const std::string &p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

void Logger::probe() {
  csv_ok = is_dir(csv_dir);
  vtk_ok = is_dir(vtk_dir);
}

void Logger::log(int64_t t, int64_t vtk_index, const std::vector<double> &u) {
  if (vtk_ok) {
    VtuWriter v(vtk_dir + "/simulate_" + std::to_string(vtk_index));
    v.append_lattice_nodes(nx, ny);
    v.append_point_data("Temperature", u);
    v.add_time_step((double)std::time(nullptr));
    v.close();
  }
  if (!csv_ok) return;
  std::ofstream out(csv_dir + "/simulate_2d.csv", std::ios_base::app);
  std::vector<double> sx(nx), sy(ny);
  const double ct = cos(2 * M_PI * (t * dt));
  for (int64_t x = 0; x < nx; ++x) sx[x] = sin(2 * M_PI * (x * dh));
  for (int64_t y = 0; y < ny; ++y) sy[y] = sin(2 * M_PI * (y * dh));
  double l2 = 0, linf = 0;
  for (int64_t x = 0; x < nx; ++x)
    for (int64_t y = 0; y < ny; ++y) {
      const double uu = u[x + y * nx], w = ct * sx[x] * sy[y];
      out << t << "," << x << "," << y << "," << uu << "," << w << "," << (uu - w) * (uu - w) << ","
          << std::abs(uu - w) << ",\n";
      l2 += (uu - w) * (uu - w);
      linf = std::max(std::abs(uu - w), linf);
    }
  out.close();
  if (test) {
    std::ofstream sc(csv_dir + "/score_2d.csv", std::ios_base::app);
    sc << t << "," << l2 << "," << linf << ",\n";
  }
}

// ---------------------------------------------------------------- loop
int run_steps(nlh_solver *s, int64_t nt, int64_t nlog, Logger &lg, bool vtk_index_is_t,
              int rank, uint64_t &elapsed_ns, int nranks, int64_t nbalance,
              const std::function<int(int64_t)> &on_balance, int64_t busy_window,
              const std::function<int(int64_t)> &on_window) {
  const bool logging = lg.enabled() && nlog > 0;
  // one rank: log steps take an asynchronous snapshot (device copy in stream
  // order, host transfer on a copy stream) and a writer thread formats the
  // files while the next steps run; several ranks gather to rank 0 (RCCL)
  const bool async_log = logging && nranks == 1;
  std::vector<double> u;
  if (logging) u.assign((size_t)(lg.nx * lg.ny), 0.0);
  std::thread writer;
  int wrc = NLH_OK;  // writer status (read after join)
  auto join_writer = [&]() -> int {
    if (writer.joinable()) writer.join();
    return wrc;
  };
  int rc = nlh_barrier(s);
  if (rc) return rc;
  const uint64_t t0 = now_ns();
  int64_t t = 0;
  bool window_open = false;  // on_window called since the last balance point
  while (t < nt) {
    int64_t last = nt - 1;  // last step of this chunk
    if (logging) {
      const int64_t next_log = (t % nlog == 0) ? t : (t / nlog + 1) * nlog;
      last = std::min(last, next_log);
    }
    const bool balancing = nbalance > 0 && on_balance;
    if (balancing) {  // load_balance after step t when t % nbalance == 0, t != 0 (:1306)
      const int64_t from = std::max<int64_t>(t, 1);
      const int64_t next_bal = (from % nbalance == 0) ? from : (from / nbalance + 1) * nbalance;
      last = std::min(last, next_bal);
      if (busy_window > 0 && on_window) {
        // the busy window: steps next_bal - busy_window + 1 .. next_bal
        // (t >= ws, not t == ws: a window as long as the interval, or one
        // that began before the chunk did, still opens -- ADVICE r5)
        const int64_t ws = std::max<int64_t>(0, next_bal - busy_window + 1);
        if (t < ws) {
          last = std::min(last, ws - 1);
        } else if (!window_open) {
          if ((rc = on_window(t)) != NLH_OK) break;
          window_open = true;
        }
      }
    }
    if ((rc = nlh_run(s, last - t + 1)) != NLH_OK) break;
    t = last + 1;
    if (balancing && last != 0 && last % nbalance == 0) {
      if ((rc = join_writer()) != NLH_OK) break;  // no snapshot across a repartition
      if ((rc = on_balance(last)) != NLH_OK) break;
      window_open = false;
    }
    if (logging && last % nlog == 0) {
      const int64_t vi = vtk_index_is_t ? last : last / nlog;
      if (async_log) {
        if ((rc = join_writer()) != NLH_OK) break;  // one snapshot in flight
        if ((rc = nlh_snapshot_begin(s)) != NLH_OK) break;
        writer = std::thread([&, last, vi] {
          wrc = nlh_snapshot_wait(s, u.data());
          if (wrc == NLH_OK) lg.log(last, vi, u);
        });
      } else {
        if ((rc = nlh_gather_field(s, 0, rank == 0 ? u.data() : nullptr)) != NLH_OK) break;
        if (rank == 0) lg.log(last, vi, u);
      }
    }
  }
  const int jr = join_writer();
  if (rc == NLH_OK) rc = jr;
  if (rc != NLH_OK) return rc;
  if ((rc = nlh_barrier(s)) != NLH_OK) return rc;
  elapsed_ns = now_ns() - t0;
  return NLH_OK;
}

bool read_partition_file(const std::string &path, int64_t &nx, int64_t &ny, int64_t &npx,
                         int64_t &npy, double &dh, std::vector<int32_t> &owner) {
  std::ifstream in(path);
  if (!in) return false;
  in >> nx >> ny >> npx >> npy >> dh;
  owner.assign((size_t)(npx * npy), 0);
  for (int64_t ix = 0; ix < npx; ++ix)
    for (int64_t iy = 0; iy < npy; ++iy) {
      int64_t px = 0, py = 0, loc = 0;
      in >> px >> py >> loc;
      if (px >= 0 && px < npx && py >= 0 && py < npy) owner[(size_t)(px + py * npx)] = (int32_t)loc;
    }
  return true;
}

int die(const char *what) {
  std::cerr << what << ": " << nlh_last_error() << std::endl;
  return 1;
}

}  // namespace nlh_drv
