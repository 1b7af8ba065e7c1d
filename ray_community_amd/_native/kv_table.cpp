// Internal key-value store of the control plane (reference: the GCS InternalKV,
// src/ray/gcs/gcs_server/gcs_kv_manager.h + store_client/in_memory_store_client.h).
//
// Namespaced byte keys -> byte values. Each namespace is an ordered map, so prefix listing and
// prefix deletion walk only the matching key range (lower_bound(prefix) .. first key without the
// prefix) instead of every key in the store. ``None`` and ``b""`` are different namespaces.
// Not thread-safe: the head calls it under its lock.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

std::string as_bytes(const py::handle& o) {
  if (py::isinstance<py::bytes>(o)) return std::string(py::reinterpret_borrow<py::bytes>(o));
  if (py::isinstance<py::str>(o)) return py::reinterpret_borrow<py::str>(o).cast<std::string>();
  throw py::type_error("kv keys, values and namespaces must be bytes or str");
}

std::string ns_key(const py::object& ns) { return ns.is_none() ? std::string("\0", 1) : "\x01" + as_bytes(ns); }

class KvTable {
 public:
  // Returns true when the key was added (false: it existed; overwritten only if ``overwrite``).
  bool put(const py::object& key, const py::object& value, bool overwrite, const py::object& ns) {
    auto& m = spaces_[ns_key(ns)];
    auto [it, added] = m.try_emplace(as_bytes(key));
    if (added || overwrite) {
      bytes_ += value_size(value) - (added ? 0 : it->second.size());
      it->second = as_bytes(value);
    }
    return added;
  }

  py::object get(const py::object& key, const py::object& ns) const {
    auto s = spaces_.find(ns_key(ns));
    if (s == spaces_.end()) return py::none();
    auto it = s->second.find(as_bytes(key));
    if (it == s->second.end()) return py::none();
    return py::bytes(it->second);
  }

  bool exists(const py::object& key, const py::object& ns) const {
    auto s = spaces_.find(ns_key(ns));
    return s != spaces_.end() && s->second.count(as_bytes(key)) != 0;
  }

  // Deletes one key, or every key starting with ``key`` when ``by_prefix``; returns the count.
  int64_t del(const py::object& key, const py::object& ns, bool by_prefix) {
    auto s = spaces_.find(ns_key(ns));
    if (s == spaces_.end()) return 0;
    auto& m = s->second;
    const std::string k = as_bytes(key);
    if (!by_prefix) {
      auto it = m.find(k);
      if (it == m.end()) return 0;
      bytes_ -= it->second.size();
      m.erase(it);
      return 1;
    }
    int64_t n = 0;
    auto it = m.lower_bound(k);
    while (it != m.end() && it->first.compare(0, k.size(), k) == 0) {
      bytes_ -= it->second.size();
      it = m.erase(it);
      ++n;
    }
    return n;
  }

  std::vector<py::bytes> keys(const py::object& prefix, const py::object& ns) const {
    std::vector<py::bytes> out;
    auto s = spaces_.find(ns_key(ns));
    if (s == spaces_.end()) return out;
    const std::string p = as_bytes(prefix);
    for (auto it = s->second.lower_bound(p); it != s->second.end() && it->first.compare(0, p.size(), p) == 0; ++it)
      out.emplace_back(it->first);
    return out;
  }

  size_t size() const {
    size_t n = 0;
    for (const auto& kv : spaces_) n += kv.second.size();
    return n;
  }

  int64_t nbytes() const { return bytes_; }

 private:
  static int64_t value_size(const py::object& v) { return (int64_t)as_bytes(v).size(); }

  std::unordered_map<std::string, std::map<std::string, std::string>> spaces_;
  int64_t bytes_ = 0;
};

}  // namespace

void register_kv_table(py::module_& m) {
  py::class_<KvTable>(m, "KvTable")
      .def(py::init<>())
      .def("put", &KvTable::put, py::arg("key"), py::arg("value"), py::arg("overwrite") = true,
           py::arg("namespace") = py::none())
      .def("get", &KvTable::get, py::arg("key"), py::arg("namespace") = py::none())
      .def("exists", &KvTable::exists, py::arg("key"), py::arg("namespace") = py::none())
      .def("delete", &KvTable::del, py::arg("key"), py::arg("namespace") = py::none(), py::arg("by_prefix") = false)
      .def("keys", &KvTable::keys, py::arg("prefix"), py::arg("namespace") = py::none())
      .def("__len__", &KvTable::size)
      .def("nbytes", &KvTable::nbytes);
}
