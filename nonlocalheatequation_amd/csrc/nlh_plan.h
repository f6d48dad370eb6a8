// nlh_plan.h -- host-only decomposition of the lattice into per-rank blocks
// and the per-step halo plan.  No device code; unit-tested on the CPU through
// nlh_halo_plan()/nlh_resolve_owner().
//
// Reference behaviour replaced:
//   tile ownership  locidx()              src/2d_nonlocal_distributed.cpp:105-110
//   --file map      param_file_input()    src/2d_nonlocal_distributed.cpp:467-488
//   neighbour set   add_neighbour_rectangle()  src/2d_nonlocal_distributed.cpp:982-992
// The reference ships WHOLE neighbour tiles through HPX actions every step
// (get_data_action, :1121-1131); here each rank holds its tiles merged into
// rectangular blocks padded by an eps-wide halo, and only the halo
// intersections move (RCCL send/recv between ranks, device copies within).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace nlh {

struct GRect {
  int64_t x0 = 0, y0 = 0, w = 0, h = 0;
  bool empty() const { return w <= 0 || h <= 0; }
};

GRect intersect(const GRect &a, const GRect &b);

struct BlockDesc {
  int32_t rank = 0;  // owner
  int32_t local = 0; // index among the owner's blocks
  GRect r;           // global node rectangle
};

struct Piece {
  int32_t src_rank = 0, dst_rank = 0;
  int32_t src_block = 0, dst_block = 0;  // indices into Plan::blocks
  GRect r;                                // global rectangle
};

struct Plan {
  std::vector<BlockDesc> blocks;  // ordered by (rank, local)
  std::vector<Piece> pieces;      // ordered by (dst_block, src_block)
};

// owner_out[i] for tile i = gx + gy*tiles_x.  owner_in == nullptr selects the
// reference default (i*nranks)/(tiles_x*tiles_y).  Returns false (and sets
// err) for an owner out of [0, nranks).
bool resolve_owner(int64_t tiles_x, int64_t tiles_y, int32_t nranks,
                   const int32_t *owner_in, std::vector<int32_t> &owner_out,
                   std::string &err);

// Merge each rank's tiles into rectangles (maximal x-runs per tile row,
// merged downwards when a run repeats) and build the halo pieces for a
// horizon `eps`.
// merge == false keeps every tile as its own block.
Plan make_plan(int64_t nx, int64_t ny, int64_t eps, int64_t tiles_x,
               int64_t tiles_y, const std::vector<int32_t> &owner, bool merge = true);

// Load-balance policy (replaces load_balance's work_realloc and DFS/BFS tile
// migration, src/2d_nonlocal_distributed.cpp:844-959).  busy[r] is rank r's
// measured busy time over one window (any unit, same for all ranks).  Each
// rank's tile quota comes from the reference's rule (:905-927): with
// d = mean - busy[r] and the rank's own time per tile tpt = busy[r]/tiles[r],
// quota = ceil(d/tpt) when d > 0.3 tpt, floor(d/tpt) when -d > 0.3 tpt, else 0.
// Tiles then move one at a time from ranks with a negative quota (never their
// last tile) to ranks with a positive one: a donor tile 4-adjacent to the
// receiver's region first (largest quota gap, then receiver-owned minus
// donor-owned neighbours, then lowest tile index), else the donor tile nearest the
// receiver's region.  A move is made only if it lowers the larger of the two
// ranks' predicted times (busy +- their own time per tile): the reference's
// quota alone hands a tile back and forth when the tiles do not divide evenly.
// Deterministic: every rank computes the same map.
// Returns the number of tiles moved; owner_out holds the new map.
// Static partitioner replacing the GMSH/METIS step of the reference's
// 2d_domain_decomposition tool (src/domain_decomposition.cpp:158-187,
// METIS_PartMeshDual on the coarse tile mesh): recursive coordinate bisection
// of the tile grid -- order the current set of tiles along the longer side of
// its bounding box and cut where the tile weight (1 each if `weight` is null)
// divides in the ratio of the parts on either side, recurse.  Parts are
// whole lines of tiles plus at most a partial line (connected staircases,
// short boundaries); parts beyond the tile count stay empty.
void partition_tiles(int64_t tiles_x, int64_t tiles_y, int32_t nparts, const double *weight,
                     std::vector<int32_t> &owner_out);

int balance_owner(int64_t tiles_x, int64_t tiles_y, int32_t nranks,
                  const std::vector<int32_t> &owner, const double *busy,
                  std::vector<int32_t> &owner_out);

// One halo piece inside the RCCL message between `me` and `peer`: me packs it
// into its send buffer for peer (dir 0) or unpacks it from its receive buffer
// from peer (dir 1), `offset` doubles into that buffer, w*h doubles long.
struct XferEntry {
  int32_t peer = 0, dir = 0;
  int32_t piece = 0;    // index into Plan::pieces
  int64_t offset = 0;   // doubles
};

// The halo pieces rank `me` exchanges with other ranks, in plan order, with
// their offsets in the per-peer messages (replaces the per-tile get_data_action
// traffic of src/2d_nonlocal_distributed.cpp:1121-1131,1156-1259).  Both
// sides walk Plan::pieces in the same order, so the offset of a piece in A's
// send buffer for B equals its offset in B's receive buffer from A (tests:
// tests/test_decomposition.py).  self_all: every piece with src_rank ==
// dst_rank == me goes to itself as well (one-rank RCCL-to-self diagnostics).
std::vector<XferEntry> exchange_layout(const Plan &plan, int32_t me, bool self_all);

}  // namespace nlh
