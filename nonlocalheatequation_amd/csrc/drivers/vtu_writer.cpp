// vtu_writer.cpp -- see vtu_writer.h.
#include "vtu_writer.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <sstream>

namespace nlh_drv {

std::string base64(const uint8_t *p, size_t n) {
  static const char *tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  out.reserve((n + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8 | p[i + 2];
    out += tbl[v >> 18 & 63];
    out += tbl[v >> 12 & 63];
    out += tbl[v >> 6 & 63];
    out += tbl[v & 63];
  }
  if (i < n) {
    uint32_t v = (uint32_t)p[i] << 16;
    if (i + 1 < n) v |= (uint32_t)p[i + 1] << 8;
    out += tbl[v >> 18 & 63];
    out += tbl[v >> 12 & 63];
    out += (i + 1 < n) ? tbl[v >> 6 & 63] : '=';
    out += '=';
  }
  return out;
}

VtuWriter::VtuWriter(const std::string &f) : fname_(f + ".vtu") {}

void VtuWriter::append_nodes(const std::vector<double> &xyz) {
  points_.assign(xyz.begin(), xyz.end());
}

void VtuWriter::append_lattice_nodes(int64_t nx, int64_t ny) {
  points_.resize((size_t)(3 * nx * ny));
  for (int64_t y = 0; y < ny; ++y)
    for (int64_t x = 0; x < nx; ++x) {
      float *p = &points_[(size_t)(3 * (x + y * nx))];
      p[0] = (float)x;
      p[1] = (float)y;
      p[2] = 0.f;
    }
}

void VtuWriter::append_point_data(const std::string &name, const std::vector<double> &v) {
  pdata_.emplace_back(name, v);
}

void VtuWriter::add_time_step(double t) {
  has_time_ = true;
  time_ = t;
}

namespace {

// appended block: base64(UInt32 byte count) + base64(payload)
std::string block(const void *data, size_t bytes) {
  const uint32_t h = (uint32_t)bytes;
  return base64(reinterpret_cast<const uint8_t *>(&h), sizeof(h)) +
         base64(reinterpret_cast<const uint8_t *>(data), bytes);
}

template <class T>
std::string range_attrs(const std::vector<T> &v, int ncomp) {
  if (v.empty()) return "";
  double lo = std::numeric_limits<double>::infinity(), hi = -lo;
  if (ncomp == 1) {
    for (auto x : v) {
      lo = std::min(lo, (double)x);
      hi = std::max(hi, (double)x);
    }
  } else {  // magnitude range, as VTK reports for vectors
    for (size_t i = 0; i + ncomp <= v.size(); i += ncomp) {
      double s = 0;
      for (int c = 0; c < ncomp; ++c) s += (double)v[i + c] * (double)v[i + c];
      s = std::sqrt(s);
      lo = std::min(lo, s);
      hi = std::max(hi, s);
    }
  }
  char buf[128];
  std::snprintf(buf, sizeof(buf), " RangeMin=\"%.17g\" RangeMax=\"%.17g\"", lo, hi);
  return buf;
}

}  // namespace

bool VtuWriter::close() {
  std::FILE *f = std::fopen(fname_.c_str(), "wb");
  if (!f) return false;
  const size_t npts = points_.size() / 3;
  std::vector<std::string> blocks;
  std::ostringstream x;
  size_t off = 0;
  auto add = [&](const std::string &b) {
    const size_t o = off;
    blocks.push_back(b);
    off += b.size();
    return o;
  };
  x << "<?xml version=\"1.0\"?>\n"
    << "<VTKFile type=\"UnstructuredGrid\" version=\"0.1\" byte_order=\"LittleEndian\" "
       "header_type=\"UInt32\">\n"
    << "  <UnstructuredGrid>\n";
  if (has_time_) {
    const size_t o = add(block(&time_, sizeof(double)));
    x << "    <FieldData>\n"
      << "      <DataArray type=\"Float64\" Name=\"TIME\" NumberOfTuples=\"1\" format=\"appended\""
      << " RangeMin=\"" << time_ << "\" RangeMax=\"" << time_ << "\" offset=\"" << o << "\"/>\n"
      << "    </FieldData>\n";
  }
  x << "    <Piece NumberOfPoints=\"" << npts << "\" NumberOfCells=\"0\">\n";
  x << "      <PointData>\n";
  for (auto &pd : pdata_) {
    const size_t o = add(block(pd.second.data(), pd.second.size() * sizeof(double)));
    x << "        <DataArray type=\"Float64\" Name=\"" << pd.first << "\" format=\"appended\""
      << range_attrs(pd.second, 1) << " offset=\"" << o << "\"/>\n";
  }
  x << "      </PointData>\n      <CellData>\n      </CellData>\n";
  {
    const size_t o = add(block(points_.data(), points_.size() * sizeof(float)));
    x << "      <Points>\n        <DataArray type=\"Float32\" Name=\"Points\" NumberOfComponents=\"3\""
      << " format=\"appended\"" << range_attrs(points_, 3) << " offset=\"" << o << "\"/>\n"
      << "      </Points>\n";
  }
  {
    const size_t oc = add(block(nullptr, 0));
    const size_t oo = add(block(nullptr, 0));
    const size_t ot = add(block(nullptr, 0));
    x << "      <Cells>\n"
      << "        <DataArray type=\"Int64\" Name=\"connectivity\" format=\"appended\" offset=\"" << oc << "\"/>\n"
      << "        <DataArray type=\"Int64\" Name=\"offsets\" format=\"appended\" offset=\"" << oo << "\"/>\n"
      << "        <DataArray type=\"UInt8\" Name=\"types\" format=\"appended\" offset=\"" << ot << "\"/>\n"
      << "      </Cells>\n";
  }
  x << "    </Piece>\n  </UnstructuredGrid>\n  <AppendedData encoding=\"base64\">\n   _";
  const std::string head = x.str();
  std::fwrite(head.data(), 1, head.size(), f);
  for (auto &b : blocks) std::fwrite(b.data(), 1, b.size(), f);
  const char *tail = "\n  </AppendedData>\n</VTKFile>\n";
  std::fwrite(tail, 1, std::strlen(tail), f);
  return std::fclose(f) == 0;
}

}  // namespace nlh_drv
