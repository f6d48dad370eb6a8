// vtu_writer.h -- dependency-free VTK XML UnstructuredGrid (.vtu) writer.
//
// Replaces rw::writer::VtkWriter (/root/reference/include/writer.{h,cpp},
// built on VTK 8.2) for the calls the solvers make: appendNodes (:30-42),
// appendPointData(name, vector<double>) (:104-117), addTimeStep (:155-161)
// and close (:163-172).  Output matches what that VTK pipeline writes: an
// UnstructuredGrid with the nodes as Points (vtkPoints default Float32), no
// cells, Float64 point data, a FieldData "TIME" array, appended data encoded
// base64 (header and payload encoded separately, UInt32 headers), no
// compression.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace nlh_drv {

class VtuWriter {
 public:
  explicit VtuWriter(const std::string &filename_no_ext);
  // node coordinates, 3 per node
  void append_nodes(const std::vector<double> &xyz);
  // lattice (x, y, 0) for an nx*ny lattice in storage order x + y*nx
  void append_lattice_nodes(int64_t nx, int64_t ny);
  void append_point_data(const std::string &name, const std::vector<double> &v);
  void add_time_step(double t);
  // writes the file; returns false if it cannot be opened
  bool close();

 private:
  std::string fname_;
  std::vector<float> points_;
  std::vector<std::pair<std::string, std::vector<double>>> pdata_;
  bool has_time_ = false;
  double time_ = 0.0;
};

std::string base64(const uint8_t *p, size_t n);

}  // namespace nlh_drv
