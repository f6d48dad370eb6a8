// comm_id_check.cpp -- CPU test harness for the drivers' RCCL-id bootstrap
// (driver_common.cpp share_comm_id, the TCP exchange that replaces HPX's
// locality bootstrap for bin/2d_nonlocal_distributed).  Run one process per
// rank with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as the
// launchers do; each performs `rounds` bootstraps back to back (successive
// batch rows).  Rank 0 sends a pseudo-random stand-in id per round (no GPU:
// share_comm_id(..., fresh = false)); every rank prints "round <i> <hex id>".
//   bin/comm_id_check [rounds=3] [seed=1]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "driver_common.h"

using namespace nlh_drv;

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 3;
  const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1u;
  const RankEnv re = rank_env();
  std::mt19937 gen(seed);
  for (int i = 0; i < rounds; ++i) {
    uint8_t id[NLH_COMM_ID_BYTES] = {0};
    if (re.rank == 0)
      for (auto &b : id) b = (uint8_t)(gen() & 0xff);
    std::string err;
    if (!share_comm_id(re, id, err, false)) {
      std::fprintf(stderr, "rank %d round %d: %s\n", re.rank, i, err.c_str());
      return 1;
    }
    std::printf("round %d ", i);
    for (auto b : id) std::printf("%02x", b);
    std::printf("\n");
    std::fflush(stdout);
  }
  return 0;
}
