// pybind11 bindings of the TF-bundle codec: actor_critic_algs_on_tensorflow_amd._C._tfbundle
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "tf_bundle.h"

namespace py = pybind11;

static py::dict entry_to_dict(const tfb::Entry& e) {
  py::dict d;
  d["key"] = e.key;
  d["dtype"] = e.dtype;
  d["shape"] = e.shape;
  d["shard_id"] = e.shard_id;
  d["offset"] = e.offset;
  d["size"] = e.size;
  d["crc32c"] = e.crc32c;
  return d;
}

PYBIND11_MODULE(_tfbundle, m) {
  m.doc() = "TensorFlow tensor-bundle (Saver V2) reader/writer, byte-compatible with TF";
  py::register_exception<tfb::FormatError>(m, "FormatError", PyExc_ValueError);
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return tfb::crc32c((const uint8_t*)s.data(), s.size());
  });
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return tfb::mask_crc(tfb::crc32c((const uint8_t*)s.data(), s.size()));
  });
  m.def("parse_index", [](py::bytes b) {
    tfb::Header h;
    std::vector<tfb::Entry> es;
    {
      std::string s = b;
      py::gil_scoped_release nogil;
      tfb::parse_index(s, &h, &es);
    }
    py::dict hd;
    hd["num_shards"] = h.num_shards;
    hd["endianness"] = h.endianness;
    hd["producer"] = h.producer;
    hd["min_consumer"] = h.min_consumer;
    py::list lst;
    for (auto& e : es) lst.append(entry_to_dict(e));
    return py::make_tuple(hd, lst);
  });
  m.def(
      "build_index",
      [](py::list entries, int num_shards, int producer) {
        tfb::Header h;
        h.num_shards = num_shards;
        h.producer = producer;
        std::vector<tfb::Entry> es;
        for (auto item : entries) {
          py::dict d = item.cast<py::dict>();
          tfb::Entry e;
          e.key = d["key"].cast<std::string>();
          e.dtype = d["dtype"].cast<int>();
          e.shape = d["shape"].cast<std::vector<int64_t>>();
          e.shard_id = d.contains("shard_id") ? d["shard_id"].cast<int32_t>() : 0;
          e.offset = d["offset"].cast<int64_t>();
          e.size = d["size"].cast<int64_t>();
          e.crc32c = d["crc32c"].cast<uint32_t>();
          es.push_back(e);
        }
        return py::bytes(tfb::build_index(h, es));
      },
      py::arg("entries"), py::arg("num_shards") = 1, py::arg("producer") = 1);
  m.def("write_bundle", [](const std::string& prefix, py::list tensors) {
    std::vector<tfb::Tensor> ts;
    for (auto item : tensors) {
      py::tuple t = item.cast<py::tuple>();
      tfb::Tensor x;
      x.key = t[0].cast<std::string>();
      x.dtype = t[1].cast<int>();
      x.shape = t[2].cast<std::vector<int64_t>>();
      x.data = t[3].cast<std::string>();
      ts.push_back(std::move(x));
    }
    py::gil_scoped_release nogil;
    tfb::write_bundle(prefix, std::move(ts));
  });
  m.def(
      "read_bundle",
      [](const std::string& prefix, bool verify) {
        std::vector<tfb::Tensor> ts;
        {
          py::gil_scoped_release nogil;
          ts = tfb::read_bundle(prefix, verify);
        }
        py::list out;
        for (auto& t : ts) out.append(py::make_tuple(t.key, t.dtype, t.shape, py::bytes(t.data)));
        return out;
      },
      py::arg("prefix"), py::arg("verify_crc") = true);
  m.def("dtype_size", &tfb::dtype_size);
}
