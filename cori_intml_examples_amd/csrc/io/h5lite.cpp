// _h5lite: a small native HDF5 reader/writer over the libhdf5 C API.
//
// The reference reads its RPV dataset through h5py (rpv.py:19-25) and writes/reads Keras
// checkpoints through Keras' h5py-based saver (rpv.py:100-101, DistHPO_mnist.ipynb:540-542).
// h5py is not available in this image, so this module provides exactly the subset those
// paths need, natively:
//   * groups (with intermediate creation), existence / kind / member listing
//   * numeric datasets (f4 f8 i1 i4 i8 u1 u4 u8) written whole, read whole or as a
//     leading-axis hyperslab [start, start+count) -- the RPV loader reads the first
//     n_samples events without touching the rest of a 1.1 GB file
//   * attributes: fixed-length byte strings (what Keras 2.2 writes: `.encode('utf8')`),
//     string arrays (`layer_names`, `weight_names`), numeric scalars/arrays; variable-length
//     strings are accepted on read (files written by newer h5py).
// Errors raise RuntimeError with the HDF5 path; libhdf5's own stderr traceback is silenced.
#include <hdf5.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

[[noreturn]] void fail(const std::string& what, const std::string& path) {
  throw std::runtime_error("h5lite: " + what + " '" + path + "'");
}

struct Hid {   // RAII for any hid_t with its matching close function
  hid_t id = -1;
  herr_t (*closer)(hid_t) = nullptr;
  Hid() = default;
  Hid(hid_t i, herr_t (*c)(hid_t)) : id(i), closer(c) {}
  Hid(const Hid&) = delete;
  Hid& operator=(const Hid&) = delete;
  Hid(Hid&& o) noexcept : id(o.id), closer(o.closer) { o.id = -1; }
  ~Hid() {
    if (id >= 0 && closer) closer(id);
  }
  operator hid_t() const { return id; }
  bool ok() const { return id >= 0; }
};

// numpy dtype char -> native HDF5 type
hid_t native_type(const py::dtype& dt) {
  const char k = dt.kind();
  const size_t n = dt.itemsize();
  if (k == 'f' && n == 4) return H5T_NATIVE_FLOAT;
  if (k == 'f' && n == 8) return H5T_NATIVE_DOUBLE;
  if (k == 'i' && n == 1) return H5T_NATIVE_INT8;
  if (k == 'i' && n == 2) return H5T_NATIVE_INT16;
  if (k == 'i' && n == 4) return H5T_NATIVE_INT32;
  if (k == 'i' && n == 8) return H5T_NATIVE_INT64;
  if (k == 'u' && n == 1) return H5T_NATIVE_UINT8;
  if (k == 'u' && n == 2) return H5T_NATIVE_UINT16;
  if (k == 'u' && n == 4) return H5T_NATIVE_UINT32;
  if (k == 'u' && n == 8) return H5T_NATIVE_UINT64;
  if (k == 'b') return H5T_NATIVE_UINT8;
  throw std::runtime_error(std::string("h5lite: unsupported numpy dtype kind '") + k + "' size " +
                           std::to_string(n));
}

// HDF5 file type -> numpy dtype (+ the native memory type to read it as)
std::pair<py::dtype, hid_t> numpy_for(hid_t ftype) {
  const H5T_class_t cls = H5Tget_class(ftype);
  const size_t n = H5Tget_size(ftype);
  if (cls == H5T_FLOAT) {
    if (n <= 4) return {py::dtype("float32"), H5T_NATIVE_FLOAT};
    return {py::dtype("float64"), H5T_NATIVE_DOUBLE};
  }
  if (cls == H5T_INTEGER) {
    const bool sgn = H5Tget_sign(ftype) == H5T_SGN_2;
    switch (n) {
      case 1: return sgn ? std::make_pair(py::dtype("int8"), H5T_NATIVE_INT8) : std::make_pair(py::dtype("uint8"), H5T_NATIVE_UINT8);
      case 2: return sgn ? std::make_pair(py::dtype("int16"), H5T_NATIVE_INT16) : std::make_pair(py::dtype("uint16"), H5T_NATIVE_UINT16);
      case 4: return sgn ? std::make_pair(py::dtype("int32"), H5T_NATIVE_INT32) : std::make_pair(py::dtype("uint32"), H5T_NATIVE_UINT32);
      default: return sgn ? std::make_pair(py::dtype("int64"), H5T_NATIVE_INT64) : std::make_pair(py::dtype("uint64"), H5T_NATIVE_UINT64);
    }
  }
  throw std::runtime_error("h5lite: unsupported HDF5 type class " + std::to_string((int)cls));
}

std::vector<std::string> split_path(const std::string& p) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    if (j > i) out.push_back(p.substr(i, j - i));
    i = j + 1;
  }
  return out;
}

// Read string attribute/dataset contents (fixed or variable length, scalar or 1-D).
py::object read_strings(hid_t obj, hid_t ftype, hid_t space, bool is_attr) {
  const int nd = H5Sget_simple_extent_ndims(space);
  if (nd < 0) throw std::runtime_error("h5lite: cannot read the dataspace rank of a string object");
  std::vector<hsize_t> dims(std::max(nd, 1), 1);
  if (nd > 0) H5Sget_simple_extent_dims(space, dims.data(), nullptr);
  size_t count = 1;
  for (int i = 0; i < nd; ++i) count *= dims[i];
  std::vector<std::string> vals;
  if (H5Tis_variable_str(ftype) > 0) {
    Hid mt(H5Tcopy(H5T_C_S1), H5Tclose);
    H5Tset_size(mt, H5T_VARIABLE);
    H5Tset_cset(mt, H5Tget_cset(ftype));
    std::vector<char*> buf(count, nullptr);
    herr_t r = is_attr ? H5Aread(obj, mt, buf.data()) : H5Dread(obj, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf.data());
    if (r < 0) throw std::runtime_error("h5lite: reading variable-length strings failed");
    for (auto* s : buf) vals.emplace_back(s ? s : "");
    H5Dvlen_reclaim(mt, space, H5P_DEFAULT, buf.data());
  } else {
    const size_t sz = H5Tget_size(ftype);
    Hid mt(H5Tcopy(H5T_C_S1), H5Tclose);
    H5Tset_size(mt, sz);
    H5Tset_strpad(mt, H5T_STR_NULLPAD);
    std::vector<char> buf(count * sz + 1, 0);
    herr_t r = is_attr ? H5Aread(obj, mt, buf.data()) : H5Dread(obj, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf.data());
    if (r < 0) throw std::runtime_error("h5lite: reading fixed-length strings failed");
    for (size_t i = 0; i < count; ++i) {
      const char* s = buf.data() + i * sz;
      vals.emplace_back(s, strnlen(s, sz));
    }
  }
  if (nd == 0) return py::bytes(vals[0]);
  py::list l;
  for (auto& v : vals) l.append(py::bytes(v));
  return std::move(l);
}

class File {
 public:
  File(const std::string& path, const std::string& mode) : path_(path) {
    H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
    if (mode == "r") {
      id_ = H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT);
    } else if (mode == "r+") {
      id_ = H5Fopen(path.c_str(), H5F_ACC_RDWR, H5P_DEFAULT);
    } else if (mode == "a") {
      id_ = H5Fis_hdf5(path.c_str()) > 0 ? H5Fopen(path.c_str(), H5F_ACC_RDWR, H5P_DEFAULT)
                                          : H5Fcreate(path.c_str(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    } else if (mode == "w") {
      id_ = H5Fcreate(path.c_str(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    } else {
      throw std::runtime_error("h5lite: bad mode " + mode);
    }
    if (id_ < 0) fail("cannot open (mode " + mode + ")", path);
  }
  ~File() { close(); }
  void close() {
    if (id_ >= 0) H5Fclose(id_);
    id_ = -1;
  }
  void flush() {
    check_open();
    H5Fflush(id_, H5F_SCOPE_GLOBAL);
  }

  bool exists(const std::string& p) {
    check_open();
    std::string cur;
    for (auto& part : split_path(p)) {
      cur += "/" + part;
      if (H5Lexists(id_, cur.c_str(), H5P_DEFAULT) <= 0) return false;
    }
    return true;
  }

  std::string kind(const std::string& p) {
    check_open();
    if (p.empty() || p == "/") return "group";
    if (!exists(p)) fail("no such object", p);
    H5O_info_t info;
    if (H5Oget_info_by_name(id_, p.c_str(), &info, H5P_DEFAULT) < 0) fail("cannot stat", p);
    if (info.type == H5O_TYPE_GROUP) return "group";
    if (info.type == H5O_TYPE_DATASET) return "dataset";
    return "other";
  }

  void create_group(const std::string& p) {
    check_open();
    std::string cur;
    for (auto& part : split_path(p)) {
      cur += "/" + part;
      if (H5Lexists(id_, cur.c_str(), H5P_DEFAULT) > 0) continue;
      Hid g(H5Gcreate2(id_, cur.c_str(), H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), H5Gclose);
      if (!g.ok()) fail("cannot create group", cur);
    }
  }

  std::vector<std::string> keys(const std::string& p) {
    check_open();
    Hid g(H5Gopen2(id_, p.empty() ? "/" : p.c_str(), H5P_DEFAULT), H5Gclose);
    if (!g.ok()) fail("no such group", p);
    std::vector<std::string> out;
    H5Literate(g, H5_INDEX_NAME, H5_ITER_INC, nullptr,
               [](hid_t, const char* name, const H5L_info_t*, void* op) -> herr_t {
                 static_cast<std::vector<std::string>*>(op)->emplace_back(name);
                 return 0;
               },
               &out);
    return out;
  }

  void write_dataset(const std::string& p, py::array arr, int gzip) {
    check_open();
    py::array a = py::array::ensure(arr, py::array::c_style);
    if (!a) fail("array not convertible", p);
    const hid_t mt = native_type(a.dtype());
    std::vector<hsize_t> dims(a.ndim());
    for (int i = 0; i < a.ndim(); ++i) dims[i] = (hsize_t)a.shape(i);
    Hid space(a.ndim() == 0 ? H5Screate(H5S_SCALAR) : H5Screate_simple(a.ndim(), dims.data(), nullptr), H5Sclose);
    if (exists(p)) H5Ldelete(id_, p.c_str(), H5P_DEFAULT);
    Hid lcpl(H5Pcreate(H5P_LINK_CREATE), H5Pclose);
    H5Pset_create_intermediate_group(lcpl, 1);
    Hid dcpl(H5Pcreate(H5P_DATASET_CREATE), H5Pclose);
    if (gzip > 0 && a.ndim() > 0 && a.size() > 0) {
      std::vector<hsize_t> chunk(dims);
      // chunk = one leading-axis row block of <= ~1 MiB
      hsize_t row = (hsize_t)a.itemsize();
      for (int i = 1; i < a.ndim(); ++i) row *= dims[i];
      chunk[0] = std::max<hsize_t>(1, std::min<hsize_t>(dims[0], (1u << 20) / std::max<hsize_t>(1, row)));
      H5Pset_chunk(dcpl, a.ndim(), chunk.data());
      H5Pset_deflate(dcpl, (unsigned)gzip);
    }
    Hid ds(H5Dcreate2(id_, p.c_str(), mt, space, lcpl, dcpl, H5P_DEFAULT), H5Dclose);
    if (!ds.ok()) fail("cannot create dataset", p);
    if (a.size() > 0 && H5Dwrite(ds, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, a.data()) < 0) fail("write failed", p);
  }

  std::vector<hsize_t> shape(const std::string& p) {
    check_open();
    Hid ds(H5Dopen2(id_, p.c_str(), H5P_DEFAULT), H5Dclose);
    if (!ds.ok()) fail("no such dataset", p);
    Hid sp(H5Dget_space(ds), H5Sclose);
    const int nd = H5Sget_simple_extent_ndims(sp);
    std::vector<hsize_t> d(nd > 0 ? nd : 0);
    if (nd > 0) H5Sget_simple_extent_dims(sp, d.data(), nullptr);
    return d;
  }

  // rows [start, start+count) along axis 0; count < 0 -> to the end
  py::object read_dataset(const std::string& p, long long start, long long count) {
    check_open();
    Hid ds(H5Dopen2(id_, p.c_str(), H5P_DEFAULT), H5Dclose);
    if (!ds.ok()) fail("no such dataset", p);
    Hid ft(H5Dget_type(ds), H5Tclose);
    Hid sp(H5Dget_space(ds), H5Sclose);
    if (H5Tget_class(ft) == H5T_STRING) return read_strings(ds, ft, sp, false);
    const int nd = H5Sget_simple_extent_ndims(sp);
    std::vector<hsize_t> dims(nd > 0 ? nd : 0);
    if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
    auto [dt, mt] = numpy_for(ft);
    if (nd == 0) {
      py::array out(dt, std::vector<py::ssize_t>{});
      if (H5Dread(ds, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, out.mutable_data()) < 0) fail("read failed", p);
      return std::move(out);
    }
    if (start < 0) start = 0;
    hsize_t n0 = dims[0];
    hsize_t s0 = std::min<hsize_t>((hsize_t)start, n0);
    hsize_t c0 = count < 0 ? n0 - s0 : std::min<hsize_t>((hsize_t)count, n0 - s0);
    std::vector<py::ssize_t> oshape(dims.begin(), dims.end());
    oshape[0] = (py::ssize_t)c0;
    py::array out(dt, oshape);
    if (c0 == 0) return std::move(out);
    std::vector<hsize_t> off(nd, 0), cnt(dims);
    off[0] = s0;
    cnt[0] = c0;
    Hid fsel(H5Scopy(sp), H5Sclose);
    H5Sselect_hyperslab(fsel, H5S_SELECT_SET, off.data(), nullptr, cnt.data(), nullptr);
    Hid msp(H5Screate_simple(nd, cnt.data(), nullptr), H5Sclose);
    herr_t r;
    {
      py::gil_scoped_release nogil;
      r = H5Dread(ds, mt, msp, fsel, H5P_DEFAULT, out.mutable_data());
    }
    if (r < 0) fail("read failed", p);
    return std::move(out);
  }

  // ---- attributes ------------------------------------------------------------------
  std::vector<std::string> attr_names(const std::string& p) {
    check_open();
    Hid o(H5Oopen(id_, p.empty() ? "/" : p.c_str(), H5P_DEFAULT), H5Oclose);
    if (!o.ok()) fail("no such object", p);
    std::vector<std::string> out;
    H5Aiterate2(o, H5_INDEX_NAME, H5_ITER_INC, nullptr,
                [](hid_t, const char* name, const H5A_info_t*, void* op) -> herr_t {
                  static_cast<std::vector<std::string>*>(op)->emplace_back(name);
                  return 0;
                },
                &out);
    return out;
  }

  // fixed-length byte-string attribute: scalar (one value) or 1-D array
  void set_attr_strings(const std::string& p, const std::string& name, const std::vector<std::string>& vals,
                        bool scalar) {
    check_open();
    Hid o(H5Oopen(id_, p.empty() ? "/" : p.c_str(), H5P_DEFAULT), H5Oclose);
    if (!o.ok()) fail("no such object", p);
    size_t sz = 1;
    for (auto& v : vals) sz = std::max(sz, v.size());
    Hid t(H5Tcopy(H5T_C_S1), H5Tclose);
    H5Tset_size(t, sz);
    H5Tset_strpad(t, H5T_STR_NULLPAD);
    hsize_t n = vals.size();
    Hid sp(scalar ? H5Screate(H5S_SCALAR) : H5Screate_simple(1, &n, nullptr), H5Sclose);
    if (H5Aexists(o, name.c_str()) > 0) H5Adelete(o, name.c_str());
    Hid a(H5Acreate2(o, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
    if (!a.ok()) fail("cannot create attribute " + name + " on", p);
    std::vector<char> buf(std::max<size_t>(1, vals.size()) * sz, 0);
    for (size_t i = 0; i < vals.size(); ++i) memcpy(buf.data() + i * sz, vals[i].data(), vals[i].size());
    if (H5Awrite(a, t, buf.data()) < 0) fail("attribute write failed " + name + " on", p);
  }

  void set_attr_array(const std::string& p, const std::string& name, py::array arr) {
    check_open();
    Hid o(H5Oopen(id_, p.empty() ? "/" : p.c_str(), H5P_DEFAULT), H5Oclose);
    if (!o.ok()) fail("no such object", p);
    py::array a = py::array::ensure(arr, py::array::c_style);
    const hid_t mt = native_type(a.dtype());
    std::vector<hsize_t> dims(a.ndim());
    for (int i = 0; i < a.ndim(); ++i) dims[i] = (hsize_t)a.shape(i);
    Hid sp(a.ndim() == 0 ? H5Screate(H5S_SCALAR) : H5Screate_simple(a.ndim(), dims.data(), nullptr), H5Sclose);
    if (H5Aexists(o, name.c_str()) > 0) H5Adelete(o, name.c_str());
    Hid at(H5Acreate2(o, name.c_str(), mt, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
    if (!at.ok()) fail("cannot create attribute " + name + " on", p);
    if (H5Awrite(at, mt, a.data()) < 0) fail("attribute write failed " + name + " on", p);
  }

  py::object get_attr(const std::string& p, const std::string& name) {
    check_open();
    Hid o(H5Oopen(id_, p.empty() ? "/" : p.c_str(), H5P_DEFAULT), H5Oclose);
    if (!o.ok()) fail("no such object", p);
    if (H5Aexists(o, name.c_str()) <= 0) throw py::key_error("h5lite: no attribute '" + name + "' on '" + p + "'");
    Hid a(H5Aopen(o, name.c_str(), H5P_DEFAULT), H5Aclose);
    Hid ft(H5Aget_type(a), H5Tclose);
    Hid sp(H5Aget_space(a), H5Sclose);
    if (H5Tget_class(ft) == H5T_STRING) return read_strings(a, ft, sp, true);
    auto [dt, mt] = numpy_for(ft);
    const int nd = H5Sget_simple_extent_ndims(sp);
    std::vector<hsize_t> dims(nd > 0 ? nd : 0);
    if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
    std::vector<py::ssize_t> shp(dims.begin(), dims.end());
    py::array out(dt, shp);
    if (H5Aread(a, mt, out.mutable_data()) < 0) fail("attribute read failed " + name + " on", p);
    return std::move(out);
  }

  bool is_open() const { return id_ >= 0; }
  const std::string& path() const { return path_; }

 private:
  void check_open() const {
    if (id_ < 0) fail("file is closed", path_);
  }
  std::string path_;
  hid_t id_ = -1;
};

}  // namespace

PYBIND11_MODULE(_h5lite, m) {
  m.doc() = "native HDF5 subset (libhdf5 C API) for RPV datasets and Keras checkpoints";
  unsigned maj = 0, mnr = 0, rel = 0;
  H5get_libversion(&maj, &mnr, &rel);
  m.attr("hdf5_version") = std::to_string(maj) + "." + std::to_string(mnr) + "." + std::to_string(rel);
  py::class_<File>(m, "File")
      .def(py::init<const std::string&, const std::string&>(), py::arg("path"), py::arg("mode") = "r")
      .def("close", &File::close)
      .def("flush", &File::flush)
      .def_property_readonly("is_open", &File::is_open)
      .def_property_readonly("path", &File::path)
      .def("exists", &File::exists)
      .def("kind", &File::kind)
      .def("create_group", &File::create_group)
      .def("keys", &File::keys, py::arg("path") = "/")
      .def("write_dataset", &File::write_dataset, py::arg("path"), py::arg("array"), py::arg("gzip") = 0)
      .def("shape", &File::shape)
      .def("read_dataset", &File::read_dataset, py::arg("path"), py::arg("start") = 0, py::arg("count") = -1)
      .def("attr_names", &File::attr_names)
      .def("set_attr_strings", &File::set_attr_strings)
      .def("set_attr_array", &File::set_attr_array)
      .def("get_attr", &File::get_attr);
}
