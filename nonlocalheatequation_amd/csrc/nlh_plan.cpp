// nlh_plan.cpp -- see nlh_plan.h.
#include "nlh_plan.h"

#include <algorithm>
#include <cstdint>
#include <cmath>
#include <cstdlib>
#include <map>

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

namespace {
bool connected(int64_t tx, const std::vector<int64_t> &tiles) {
  if (tiles.size() <= 1) return true;
  std::vector<int64_t> sorted(tiles);
  std::sort(sorted.begin(), sorted.end());
  auto has = [&](int64_t t) { return std::binary_search(sorted.begin(), sorted.end(), t); };
  std::vector<int64_t> stack{sorted[0]}, seen{sorted[0]};
  while (!stack.empty()) {
    const int64_t t = stack.back();
    stack.pop_back();
    const int64_t x = t % tx;
    const int64_t nb[4] = {x > 0 ? t - 1 : -1, x + 1 < tx ? t + 1 : -1, t - tx, t + tx};
    for (int64_t u : nb) {
      if (u < 0 || !has(u) || std::find(seen.begin(), seen.end(), u) != seen.end()) continue;
      seen.push_back(u);
      stack.push_back(u);
    }
  }
  return seen.size() == sorted.size();
}

// bisect a set of tiles: order it along the longer side of its bounding box
// (the other coordinate second, so a prefix is whole lines plus part of one,
// a staircase that stays connected) and cut where the weight divides in the
// ratio of the parts on either side
void rcb(int64_t tx, const double *w, std::vector<int64_t> tiles, int32_t r0, int32_t nr,
         std::vector<int32_t> &o) {
  if (nr <= 1 || tiles.size() <= 1) {
    for (int64_t t : tiles) o[t] = r0;
    return;
  }
  int64_t x0 = tx, x1 = -1, y0 = INT64_MAX, y1 = -1;
  for (int64_t t : tiles) {
    x0 = std::min(x0, t % tx);
    x1 = std::max(x1, t % tx);
    y0 = std::min(y0, t / tx);
    y1 = std::max(y1, t / tx);
  }
  const bool cols = (x1 - x0) >= (y1 - y0);  // cut across the longer side
  std::sort(tiles.begin(), tiles.end(), [&](int64_t a, int64_t b) {
    const int64_t pa = cols ? a % tx : a / tx, pb = cols ? b % tx : b / tx;
    if (pa != pb) return pa < pb;
    return (cols ? a / tx : a % tx) < (cols ? b / tx : b % tx);
  });
  const int32_t nl = nr / 2;
  double total = 0.0;
  for (int64_t t : tiles) total += w ? w[t] : 1.0;
  const double target = total * nl / nr;
  size_t cut = 1;
  double cum = w ? w[tiles[0]] : 1.0, best = std::fabs(cum - target);
  for (size_t k = 2; k < tiles.size(); ++k) {  // first k tiles to the lower parts
    cum += w ? w[tiles[k - 1]] : 1.0;
    const double d = std::fabs(cum - target);
    if (d < best) {
      best = d;
      cut = k;
    }
  }
  std::vector<int64_t> lo(tiles.begin(), tiles.begin() + cut), hi(tiles.begin() + cut, tiles.end());
  // the cut line is split; if taking its low end leaves either side in two
  // pieces, take its high end instead (same count, so the same weights with
  // unit weights)
  if (!(connected(tx, lo) && connected(tx, hi))) {
    auto line = [&](int64_t t) { return cols ? t % tx : t / tx; };
    const int64_t L = line(tiles[cut]);
    size_t b = cut, e = cut;
    while (b > 0 && line(tiles[b - 1]) == L) --b;
    while (e < tiles.size() && line(tiles[e]) == L) ++e;
    if (b < cut) {  // m = cut - b tiles of line L go low: try the top m instead
      std::vector<int64_t> lo2(tiles.begin(), tiles.begin() + b), hi2;
      lo2.insert(lo2.end(), tiles.begin() + (e - (cut - b)), tiles.begin() + e);
      hi2.insert(hi2.end(), tiles.begin() + b, tiles.begin() + (e - (cut - b)));
      hi2.insert(hi2.end(), tiles.begin() + e, tiles.end());
      if (connected(tx, lo2) && connected(tx, hi2)) {
        lo.swap(lo2);
        hi.swap(hi2);
      }
    }
  }
  rcb(tx, w, lo, r0, nl, o);
  rcb(tx, w, hi, r0 + nl, nr - nl, o);
}
}  // namespace

void partition_tiles(int64_t tiles_x, int64_t tiles_y, int32_t nparts, const double *weight,
                     std::vector<int32_t> &owner_out) {
  owner_out.assign((size_t)(tiles_x * tiles_y), 0);
  std::vector<int64_t> all((size_t)(tiles_x * tiles_y));
  for (size_t i = 0; i < all.size(); ++i) all[i] = (int64_t)i;
  rcb(tiles_x, weight, all, 0, std::max<int32_t>(1, nparts), owner_out);
}

int balance_owner(int64_t tiles_x, int64_t tiles_y, int32_t nranks,
                  const std::vector<int32_t> &owner, const double *busy,
                  std::vector<int32_t> &owner_out) {
  const int64_t T = tiles_x * tiles_y;
  owner_out = owner;
  if (nranks < 2 || T < 2) return 0;
  std::vector<int64_t> n(nranks, 0);
  for (int64_t i = 0; i < T; ++i) ++n[owner[i]];
  double total = 0.0;
  for (int r = 0; r < nranks; ++r) total += busy[r] > 0 ? busy[r] : 0.0;
  if (!(total > 0.0)) return 0;
  const double mean = total / nranks;
  // quota per rank, the reference's work_realloc (:905-927); a rank without
  // tiles is priced at the job's mean time per tile
  std::vector<int64_t> w(nranks, 0);
  std::vector<double> P(nranks), tp(nranks);  // predicted busy time, time per tile
  for (int r = 0; r < nranks; ++r) {
    const double b = busy[r] > 0 ? busy[r] : 0.0;
    const double tpt = n[r] > 0 && b > 0 ? b / (double)n[r] : total / (double)T;
    P[r] = b;
    tp[r] = tpt;
    const double d = mean - b;
    if (d > 0 && d > 0.3 * tpt)
      w[r] = (int64_t)std::ceil(d / tpt);
    else if (d < 0 && -d > 0.3 * tpt)
      w[r] = (int64_t)std::floor(d / tpt);
  }
  std::vector<int32_t> &o = owner_out;
  auto nbrs = [&](int64_t t, int64_t out[4]) {
    const int64_t gx = t % tiles_x, gy = t / tiles_x;
    int k = 0;
    if (gx > 0) out[k++] = t - 1;
    if (gx + 1 < tiles_x) out[k++] = t + 1;
    if (gy > 0) out[k++] = t - tiles_x;
    if (gy + 1 < tiles_y) out[k++] = t + tiles_x;
    return k;
  };
  int moved = 0;
  for (int64_t guard = 0; guard < T * nranks; ++guard) {
    // adjacent moves: (quota gap, receiver-owned neighbours, -tile index)
    int64_t bt = -1;
    int br = -1;
    int64_t bgap = 0, bown = -8;
    for (int64_t t = 0; t < T; ++t) {
      const int d = o[t];
      if (w[d] >= 0 || n[d] <= 1) continue;
      int64_t nb[4];
      const int k = nbrs(t, nb);
      for (int j = 0; j < k; ++j) {
        const int r = o[nb[j]];
        if (r == d || w[r] <= 0 || !(P[r] + tp[r] < P[d])) continue;
        int64_t own = 0;  // receiver-owned minus donor-owned neighbours: keep regions compact
        for (int q = 0; q < k; ++q) own += (o[nb[q]] == r) - (o[nb[q]] == d);
        const int64_t gap = w[r] - w[d];
        if (bt < 0 || gap > bgap || (gap == bgap && own > bown)) {
          bt = t;
          br = r;
          bgap = gap;
          bown = own;
        }
      }
    }
    if (bt < 0) {
      // no donor borders a receiver: the pair with the largest quota gap,
      // donor tile nearest (Manhattan) the receiver's tiles
      int bd = -1;
      for (int d = 0; d < nranks; ++d)
        if (w[d] < 0 && n[d] > 1 && (bd < 0 || w[d] < w[bd])) bd = d;
      for (int r = 0; r < nranks; ++r)
        if (w[r] > 0 && (br < 0 || w[r] > w[br])) br = r;
      if (bd < 0 || br < 0 || !(P[br] + tp[br] < P[bd])) break;
      // distance of every tile to the receiver's nearest tile: one
      // multi-source BFS over the tile grid (= the Manhattan distance, the grid
      // has no obstacles), O(T) per move instead of donor x receiver pairs
      std::vector<int64_t> dist((size_t)T, -1), queue;
      queue.reserve((size_t)T);
      for (int64_t t = 0; t < T; ++t)
        if (o[t] == br) {
          dist[t] = 0;
          queue.push_back(t);
        }
      for (size_t h = 0; h < queue.size(); ++h) {
        int64_t nb[4];
        const int k = nbrs(queue[h], nb);
        for (int j = 0; j < k; ++j)
          if (dist[nb[j]] < 0) {
            dist[nb[j]] = dist[queue[h]] + 1;
            queue.push_back(nb[j]);
          }
      }
      int64_t bdist = -1;
      for (int64_t t = 0; t < T; ++t) {
        if (o[t] != bd) continue;
        const int64_t dt = n[br] ? dist[t] : 0;  // a receiver without tiles: any donor tile
        if (bdist < 0 || dt < bdist) {
          bdist = dt;
          bt = t;
        }
      }
      if (bt < 0) break;
    }
    const int d = o[bt];
    P[d] -= tp[d];
    P[br] += tp[br];
    o[bt] = br;
    ++w[d];
    --w[br];
    --n[d];
    ++n[br];
    ++moved;
  }
  return moved;
}

std::vector<XferEntry> exchange_layout(const Plan &plan, int32_t me, bool self_all) {
  std::vector<XferEntry> out;
  std::map<int32_t, int64_t> soff, roff;
  for (size_t i = 0; i < plan.pieces.size(); ++i) {
    const Piece &pc = plan.pieces[i];
    const bool remote = pc.src_rank != pc.dst_rank || (self_all && pc.src_rank == me);
    if (!remote) continue;
    const int64_t n = pc.r.w * pc.r.h;
    if (pc.src_rank == me) {
      out.push_back({pc.dst_rank, 0, (int32_t)i, soff[pc.dst_rank]});
      soff[pc.dst_rank] += n;
    }
    if (pc.dst_rank == me) {
      out.push_back({pc.src_rank, 1, (int32_t)i, roff[pc.src_rank]});
      roff[pc.src_rank] += n;
    }
  }
  return out;
}

}  // namespace nlh
