// 2d_domain_decomposition -- counterpart of the reference's GMSH/METIS tool
// (/root/reference/src/domain_decomposition.cpp) that writes the --file
// partition file 2d_nonlocal_distributed reads.
//
//   2d_domain_decomposition mesh out_filename number_compute_nodes
//
// mesh: a GMSH 4.1 ASCII .msh quad mesh (nodes + 4-node quadrangles, the input
// the reference opens with gmsh::open, :64-71), or "MXxMY:DH" naming the fine
// mesh directly (MX x MY cells of size DH) -- GMSH itself is not needed.
// Same console dialogue (:108-147: mesh size, then the coarse grain sizes on
// stdin, which must divide the mesh size), same output file (write_mesh,
// :31-50: "mx/npx my/npy npx npy dh", then "idx idy part" with idx outer).
// The METIS_PartMeshDual step (:158-187) is replaced by nlh_partition_tiles
// (recursive coordinate bisection of the tile grid, host-only, no GPU).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "nlh.h"

namespace {

// fine mesh extent and spacing from a GMSH 4.1 ASCII file: dh from the first
// quadrangle's first two nodes and the bounding box of all quadrangle nodes
// (:76-106)
bool read_msh(const std::string &path, long &mx, long &my, double &dh, std::string &err) {
  std::ifstream in(path);
  if (!in) {
    err = "cannot open " + path;
    return false;
  }
  std::unordered_map<long, std::pair<double, double>> xy;
  std::vector<long> quads;  // 4 node tags per quadrangle
  std::string line;
  while (std::getline(in, line)) {
    if (line.rfind("$MeshFormat", 0) == 0) {
      double ver = 0;
      int ft = 0, ds = 0;
      in >> ver >> ft >> ds;
      if (ver < 4.0 || ft != 0) {
        err = "only GMSH 4.x ASCII meshes are read";
        return false;
      }
    } else if (line.rfind("$Nodes", 0) == 0) {
      long nblocks = 0, nnodes = 0, mn = 0, mxg = 0;
      in >> nblocks >> nnodes >> mn >> mxg;
      for (long b = 0; b < nblocks; ++b) {
        int edim = 0, etag = 0, param = 0;
        long n = 0;
        in >> edim >> etag >> param >> n;
        std::vector<long> tags(n);
        for (auto &t : tags) in >> t;
        for (long i = 0; i < n; ++i) {
          double x, y, z;
          in >> x >> y >> z;
          for (int k = 0; k < param * edim; ++k) {
            double u;
            in >> u;
          }
          xy[tags[i]] = {x, y};
        }
      }
    } else if (line.rfind("$Elements", 0) == 0) {
      long nblocks = 0, nel = 0, mn = 0, mxg = 0;
      in >> nblocks >> nel >> mn >> mxg;
      for (long b = 0; b < nblocks; ++b) {
        int edim = 0, etag = 0, etype = 0;
        long n = 0;
        in >> edim >> etag >> etype >> n;
        std::getline(in, line);
        for (long i = 0; i < n; ++i) {
          std::getline(in, line);
          if (etype != 3) continue;  // 4-node quadrangle
          std::istringstream ls(line);
          long tag, a[4];
          ls >> tag >> a[0] >> a[1] >> a[2] >> a[3];
          quads.insert(quads.end(), a, a + 4);
        }
      }
    }
  }
  if (quads.empty()) {
    err = "no quadrangle elements in " + path;
    return false;
  }
  auto at = [&](long tag) { return xy.at(tag); };
  dh = std::max(std::abs(at(quads[0]).first - at(quads[1]).first),
                std::abs(at(quads[0]).second - at(quads[1]).second));
  double minx = 1e300, maxx = -1e300, miny = 1e300, maxy = -1e300;
  for (long t : quads) {
    const auto p = at(t);
    minx = std::min(minx, p.first);
    maxx = std::max(maxx, p.first);
    miny = std::min(miny, p.second);
    maxy = std::max(maxy, p.second);
  }
  if (!(dh > 0)) {
    err = "degenerate quadrangle";
    return false;
  }
  mx = std::lround((maxx - minx) / dh);
  my = std::lround((maxy - miny) / dh);
  return true;
}

bool parse_spec(const std::string &s, long &mx, long &my, double &dh) {
  char x = 0, c = 0;
  std::istringstream in(s);
  return (in >> mx >> x >> my >> c >> dh) && x == 'x' && c == ':' && mx > 0 && my > 0 && dh > 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 4) {
    std::cout << "Usage: " << argv[0] << " mesh_filename out_filename number_compute_nodes" << std::endl;
    return 0;
  }
  const std::string mesh = argv[1], out_name = argv[2];
  const long nodes = std::atol(argv[3]);
  long mx = 0, my = 0;
  double dh = 0;
  std::string err;
  if (!parse_spec(mesh, mx, my, dh) && !read_msh(mesh, mx, my, dh, err)) {
    std::cerr << err << std::endl;
    return 1;
  }
  std::cout << "\nSize of mesh is as follows:\n";
  std::cout << "x dimension : " << mx << "\ny dimension : " << my;
  std::cout << "\n\nNote:" << std::endl;
  std::cout << "Enter coarse grain size as a divisor for size of mesh along repective dimension" << std::endl;
  std::cout << "1 <= Coarse grain size on x-dimension <= Mesh size on x-dimension" << std::endl;
  std::cout << "1 <= Coarse grain size on y-dimension <= Mesh size on y-dimension" << std::endl;
  long npx = 0, npy = 0;
  std::cout << "\n\nEnter coarse mesh size along x-dimension" << std::endl;
  std::cin >> npx;
  if (npx < 1 || mx % npx != 0) {
    std::cout << "Mesh size along x direction not divisible by the coarse grain size in x-direction" << std::endl;
    return 0;
  }
  npx = mx / npx;
  std::cout << "\n\nEnter coarse mesh size along y-dimension" << std::endl;
  std::cin >> npy;
  if (npy < 1 || my % npy != 0) {
    std::cout << "Mesh size along y direction not divisible by the coarse grain size in y-direction" << std::endl;
    return 0;
  }
  npy = my / npy;

  std::vector<int32_t> parts((size_t)(npx * npy), 0);
  if (nodes >= 2 && nlh_partition_tiles(npx, npy, (int32_t)nodes, nullptr, parts.data()) != NLH_OK) {
    std::cerr << "nlh_partition_tiles: " << nlh_last_error() << std::endl;
    return 1;
  }
  std::ofstream out(out_name);
  if (out) {
    out << mx / npx << " " << my / npy << " " << npx << " " << npy << " " << dh << std::endl;
    for (long ix = 0; ix < npx; ++ix)
      for (long iy = 0; iy < npy; ++iy) out << ix << " " << iy << " " << parts[ix + iy * npx] << std::endl;
  }
  return 0;
}
