// driver_common.h -- shared pieces of the drop-in drivers 2d_nonlocal_serial,
// 2d_nonlocal_async and 2d_nonlocal_distributed.
//
// Replaces, for the driver surface only:
//   hpx::program_options / hpx::init  -> Options (same flag names, defaults,
//                                         "--name value" / "--name=value",
//                                         bare flags; --hpx:* accepted and
//                                         ignored)
//   print_time_results (include/print_time_results.hpp:19-97) -> print_time_*
//   HPX localities -> one process per GPU; rank/size from the launcher's
//                     environment, RCCL unique id shared over a TCP socket
//                     (MASTER_ADDR / MASTER_PORT, as torch.distributed.run sets)
//   CSV logging (src/2d_nonlocal_serial.cpp:149-177, async :214-284)
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "nlh.h"

namespace nlh_drv {

class Options {
 public:
  void flag(const std::string &name);  // presence-only option
  void opt(const std::string &name, const std::string &def);
  // returns false and sets err on an unknown option or a missing value
  bool parse(int argc, char **argv, std::string &err);
  bool count(const std::string &name) const;  // flag given
  std::string str(const std::string &name) const;
  bool as_bool(const std::string &name) const;
  int64_t as_i64(const std::string &name) const;
  uint64_t as_u64(const std::string &name) const;
  double as_double(const std::string &name) const;

 private:
  std::map<std::string, bool> flags_;
  std::map<std::string, std::string> vals_;
};

void print_banner(const char *argv0);

// include/print_time_results.hpp:64-81 (serial / async)
void print_time_results(uint64_t threads, uint64_t elapsed_ns, uint64_t nx, uint64_t ny,
                        uint64_t nt, bool header);
// include/print_time_results.hpp:19-41 (distributed)
void print_time_results(uint32_t localities, uint64_t threads, uint64_t elapsed_ns,
                        uint64_t nx, uint64_t ny, uint64_t npx, uint64_t npy, uint64_t nt,
                        bool header);

// include/print_time_results.hpp:84-99 (1d)
void print_time_results(uint64_t threads, uint64_t elapsed_ns, uint64_t nx, uint64_t nt, bool header);

uint64_t now_ns();

struct RankEnv {
  int rank = 0, nranks = 1, local_rank = 0;
};
RankEnv rank_env();
// RCCL unique id from rank 0 to every rank over TCP (MASTER_ADDR,
// MASTER_PORT + 1); fresh == false: rank 0 sends the id it was given instead
// of a new RCCL id (tools/comm_id_check.cpp tests the bootstrap without a GPU)
bool share_comm_id(const RankEnv &re, uint8_t id[NLH_COMM_ID_BYTES], std::string &err, bool fresh = true);

int kernel_from_name(const std::string &s);

// --kernel auto in test mode: the drivers print the
// reference's l2 / linfinity, which the FAST kernels reproduce only to the
// L2 contract of include/nlh.h.  Where the EXACT kernel's whole run is cheap
// -- nx*ny*nt*N(eps) <= kDriverExactTerms disk terms, well under a second on
// one MI355X -- AUTO becomes EXACT, so the printed numbers are the
// reference's own order bit for bit (every row of the reference's batch
// files).  Returns the kernel to request.
constexpr double kDriverExactTerms = 2e11;
int driver_kernel(const nlh_params &p, int64_t nt);
// after nlh_create: when the run prints test-mode errors from a FAST kernel
// that --kernel auto chose, one line on stderr names the kernel and the
// contract its l2 follows
void note_fast_test_kernel(nlh_solver *s, const nlh_params &p, int requested, bool print);
// --influence constant|linear -> enum nlh_influence (-1 if unknown)
int influence_from_name(const std::string &s);

// host w(x, y, t) exactly as the reference (src/2d_nonlocal_serial.cpp:207-210)
double w_exact(int64_t x, int64_t y, int64_t t, double dt, double dh);

// Logger for the reference's ../out_csv and ../out_vtk outputs.  Files are
// written only when the directory exists (the reference's streams fail
// silently otherwise).
struct Logger {
  int64_t nx = 0, ny = 0;
  double dt = 0, dh = 0;
  bool test = false;
  bool csv_ok = false, vtk_ok = false;
  std::string csv_dir = "../out_csv", vtk_dir = "../out_vtk";
  void probe();
  bool enabled() const { return csv_ok || vtk_ok; }
  // u_next = S[next] after step t; w evaluated at t (reference off-by-one,
  // :149-162); vtk file index `vtk_index`
  void log(int64_t t, int64_t vtk_index, const std::vector<double> &u_next);
};

// Print "l2: .. linfinity: .." and optionally the comparison lines.
void print_errors(double l2, double linf);

// The reference's do_work time loop with its logging cadence: after step t,
// if t % nlog == 0, log S[next] (serial names the VTK file t/nlog, the tiled
// solvers t).  Steps between log points are enqueued back to back.  Collective
// when nranks > 1 (the field is gathered to rank 0 for logging); with one
// rank the log steps snapshot the field asynchronously (nlh_snapshot_begin)
// and a writer thread writes the files while the following steps run.
// Returns NLH_OK and the wall time of the loop (all ranks finished, the last
// files written) in elapsed_ns.
// nbalance > 0: on_balance(t) runs after step t whenever t % nbalance == 0
// and t != 0 (the reference's load_balance cadence, src/2d_nonlocal_
// distributed.cpp:1306-1309), before that step's log.
// busy_window > 0 (with nbalance): on_window(t) runs before step t = the
// first of the busy_window steps that precede each balance point -- the
// driver switches busy timing (nlh_kernel_timing mode 2, which serialises a
// pass's kernels) on there and off again after the balance, so the other
// steps keep the overlapped exchange schedule.
int run_steps(nlh_solver *s, int64_t nt, int64_t nlog, Logger &lg, bool vtk_index_is_t,
              int rank, uint64_t &elapsed_ns, int nranks = 1, int64_t nbalance = 0,
              const std::function<int(int64_t)> &on_balance = {}, int64_t busy_window = 0,
              const std::function<int(int64_t)> &on_window = {});

// Read the reference's --file partition file (src/2d_nonlocal_distributed.cpp:
// 467-488): "nx ny npx npy dh" then npx*npy lines "px py owner", px outer.
// Returns false if the file cannot be opened (the reference then keeps the
// command-line values).
bool read_partition_file(const std::string &path, int64_t &nx, int64_t &ny, int64_t &npx,
                         int64_t &npy, double &dh, std::vector<int32_t> &owner);

int die(const char *what);  // prints nlh_last_error() and returns 1

}  // namespace nlh_drv
