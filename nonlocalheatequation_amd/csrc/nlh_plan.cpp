// nlh_plan.cpp -- see nlh_plan.h.
#include "nlh_plan.h"

#include <algorithm>

namespace nlh {

GRect intersect(const GRect &a, const GRect &b) {
  GRect r;
  r.x0 = std::max(a.x0, b.x0);
  r.y0 = std::max(a.y0, b.y0);
  r.w = std::min(a.x0 + a.w, b.x0 + b.w) - r.x0;
  r.h = std::min(a.y0 + a.h, b.y0 + b.h) - r.y0;
  if (r.w < 0) r.w = 0;
  if (r.h < 0) r.h = 0;
  return r;
}

bool resolve_owner(int64_t tiles_x, int64_t tiles_y, int32_t nranks,
                   const int32_t *owner_in, std::vector<int32_t> &owner_out,
                   std::string &err) {
  const int64_t T = tiles_x * tiles_y;
  owner_out.assign((size_t)T, 0);
  for (int64_t i = 0; i < T; ++i) {
    int64_t o = owner_in ? owner_in[i] : (i * nranks) / T;  // locidx()
    if (o < 0 || o >= nranks) {
      err = "tile " + std::to_string(i) + " owner " + std::to_string(o) +
            " outside [0, " + std::to_string(nranks) + ")";
      return false;
    }
    owner_out[(size_t)i] = (int32_t)o;
  }
  return true;
}

Plan make_plan(int64_t nx, int64_t ny, int64_t eps, int64_t tiles_x,
               int64_t tiles_y, const std::vector<int32_t> &owner, bool merge) {
  Plan plan;
  const int64_t tw = nx / tiles_x, th = ny / tiles_y;
  int32_t nranks = 0;
  for (int32_t o : owner) nranks = std::max(nranks, o + 1);

  for (int32_t rank = 0; rank < nranks; ++rank) {
    // open rectangles in tile units: {gx0, gx1, gy0, gy1}
    struct TR { int64_t gx0, gx1, gy0, gy1; };
    std::vector<TR> done, open;
    for (int64_t gy = 0; gy < tiles_y; ++gy) {
      std::vector<TR> runs;
      for (int64_t gx = 0; gx < tiles_x;) {
        if (owner[(size_t)(gx + gy * tiles_x)] != rank) { ++gx; continue; }
        int64_t e = gx + 1;
        while (merge && e < tiles_x && owner[(size_t)(e + gy * tiles_x)] == rank) ++e;
        runs.push_back({gx, e, gy, gy + 1});
        gx = e;
      }
      std::vector<TR> next_open;
      for (auto &o : open) {
        auto it = std::find_if(runs.begin(), runs.end(), [&](const TR &r) {
          return r.gx0 == o.gx0 && r.gx1 == o.gx1;
        });
        if (merge && it != runs.end()) {
          TR m = o;
          m.gy1 = gy + 1;
          next_open.push_back(m);
          runs.erase(it);
        } else {
          done.push_back(o);
        }
      }
      for (auto &r : runs) next_open.push_back(r);
      open.swap(next_open);
    }
    for (auto &o : open) done.push_back(o);
    std::sort(done.begin(), done.end(), [](const TR &a, const TR &b) {
      return a.gy0 != b.gy0 ? a.gy0 < b.gy0 : a.gx0 < b.gx0;
    });
    int32_t local = 0;
    for (auto &d : done) {
      BlockDesc b;
      b.rank = rank;
      b.local = local++;
      b.r.x0 = d.gx0 * tw;
      b.r.y0 = d.gy0 * th;
      b.r.w = (d.gx1 - d.gx0) * tw;
      b.r.h = (d.gy1 - d.gy0) * th;
      plan.blocks.push_back(b);
    }
  }

  const GRect dom{0, 0, nx, ny};
  for (size_t di = 0; di < plan.blocks.size(); ++di) {
    const GRect &B = plan.blocks[di].r;
    GRect halo{B.x0 - eps, B.y0 - eps, B.w + 2 * eps, B.h + 2 * eps};
    halo = intersect(halo, dom);
    for (size_t si = 0; si < plan.blocks.size(); ++si) {
      if (si == di) continue;
      GRect r = intersect(plan.blocks[si].r, halo);
      if (r.empty()) continue;
      Piece p;
      p.src_rank = plan.blocks[si].rank;
      p.dst_rank = plan.blocks[di].rank;
      p.src_block = (int32_t)si;
      p.dst_block = (int32_t)di;
      p.r = r;
      plan.pieces.push_back(p);
    }
  }
  return plan;
}

}  // namespace nlh
