// Object reference table of the head's control plane: who holds every object, how often it is
// pinned, and which node's store has its value.
//
// Reference parity: the ownership-based reference counting of the reference's core worker
// (src/ray/core_worker/reference_count.h: ReferenceCounter -- per-object local/submitted/borrower
// references, OnRefRemoved -> delete) and the object directory's node locations
// (src/ray/object_manager/ownership_object_directory.h). Here one table in the head covers all
// of it: a "holder" is a process or handle key (driver, "w:<worker>", caller ids) that keeps an
// object alive; a "pin" is an anonymous count (objects nested inside other objects, in-flight
// task arguments). An object is referenced while it has a holder or a positive pin count.
//
// Design: holder keys and node ids are interned to 32-bit ids; each object keeps a small vector
// of holder ids (almost always 1-3, so a linear scan beats a hash set), a pin count and a node id;
// a reverse index holder -> objects makes a process death cost O(objects it held) instead of a
// scan over every object in the cluster (head.py _drop_holder_everywhere), and a node index makes
// node loss O(objects on that node). All operations are O(1) amortised except drop_holder /
// objects_on_node (linear in their result). Not thread-safe: the head calls it under its lock.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace {

class Interner {
 public:
  uint32_t id(const std::string& s) {
    auto it = ids_.find(s);
    if (it != ids_.end()) return it->second;
    const uint32_t v = (uint32_t)names_.size();
    names_.push_back(s);
    ids_.emplace(s, v);
    return v;
  }
  bool find(const std::string& s, uint32_t& v) const {
    auto it = ids_.find(s);
    if (it == ids_.end()) return false;
    v = it->second;
    return true;
  }
  const std::string& name(uint32_t v) const { return names_[v]; }

 private:
  std::unordered_map<std::string, uint32_t> ids_;
  std::vector<std::string> names_;
};

constexpr uint32_t kNoNode = 0xffffffffu;

struct Rec {
  std::vector<uint32_t> holders;
  int64_t pins = 0;
  uint32_t node = kNoNode;
};

class RefTable {
 public:
  bool add(const py::bytes& oid) { return objs_.try_emplace(std::string(oid)).second; }

  bool contains(const py::bytes& oid) const { return objs_.count(std::string(oid)) != 0; }

  size_t size() const { return objs_.size(); }

  // Forget the object entirely (its value was freed): drops it from every index.
  void erase(const py::bytes& oid) {
    auto it = objs_.find(std::string(oid));
    if (it == objs_.end()) return;
    for (uint32_t h : it->second.holders) unindex_holder(h, it->first);
    if (it->second.node != kNoNode) unindex_node(it->second.node, it->first);
    objs_.erase(it);
  }

  // Returns true if the key was not a holder yet. Creates the record if needed.
  bool add_holder(const py::bytes& oid, const std::string& key) {
    const std::string o(oid);
    Rec& r = objs_[o];
    const uint32_t h = keys_.id(key);
    for (uint32_t x : r.holders)
      if (x == h) return false;
    r.holders.push_back(h);
    by_holder_[h].insert(o);
    return true;
  }

  // Removes one holder; returns true when the object is now unreferenced (no holder, pins <= 0).
  bool remove_holder(const py::bytes& oid, const std::string& key) {
    uint32_t h;
    if (!keys_.find(key, h)) return unreferenced(oid);
    const std::string o(oid);
    auto it = objs_.find(o);
    if (it == objs_.end()) return false;
    auto& hs = it->second.holders;
    for (size_t i = 0; i < hs.size(); ++i) {
      if (hs[i] == h) {
        hs[i] = hs.back();
        hs.pop_back();
        unindex_holder(h, o);
        break;
      }
    }
    return hs.empty() && it->second.pins <= 0;
  }

  bool has_holder(const py::bytes& oid, const std::string& key) const {
    uint32_t h;
    if (!keys_.find(key, h)) return false;
    auto it = objs_.find(std::string(oid));
    if (it == objs_.end()) return false;
    for (uint32_t x : it->second.holders)
      if (x == h) return true;
    return false;
  }

  // pin(+n) / unpin(-n); returns true when the object is now unreferenced. Creates the record
  // (the head only pins objects it tracks, so no separate add() is needed on the hot path).
  bool pin(const py::bytes& oid, int64_t n) {
    Rec& r = objs_[std::string(oid)];
    r.pins += n;
    return r.holders.empty() && r.pins <= 0;
  }

  int64_t pins(const py::bytes& oid) const {
    auto it = objs_.find(std::string(oid));
    return it == objs_.end() ? 0 : it->second.pins;
  }

  size_t num_holders(const py::bytes& oid) const {
    auto it = objs_.find(std::string(oid));
    return it == objs_.end() ? 0 : it->second.holders.size();
  }

  std::vector<std::string> holders(const py::bytes& oid) const {
    std::vector<std::string> out;
    auto it = objs_.find(std::string(oid));
    if (it != objs_.end())
      for (uint32_t h : it->second.holders) out.push_back(keys_.name(h));
    return out;
  }

  bool referenced(const py::bytes& oid) const {
    auto it = objs_.find(std::string(oid));
    return it != objs_.end() && (!it->second.holders.empty() || it->second.pins > 0);
  }

  bool unreferenced(const py::bytes& oid) const {
    auto it = objs_.find(std::string(oid));
    return it != objs_.end() && it->second.holders.empty() && it->second.pins <= 0;
  }

  // Every holder and pin dropped (the object is being lost/recomputed from scratch).
  void clear_refs(const py::bytes& oid) {
    const std::string o(oid);
    auto it = objs_.find(o);
    if (it == objs_.end()) return;
    for (uint32_t h : it->second.holders) unindex_holder(h, o);
    it->second.holders.clear();
    it->second.pins = 0;
  }

  // A holder went away (process death, client disconnect): remove it from every object it held
  // and return the objects left unreferenced by that.
  std::vector<py::bytes> drop_holder(const std::string& key) {
    std::vector<py::bytes> freed;
    uint32_t h;
    if (!keys_.find(key, h)) return freed;
    auto bh = by_holder_.find(h);
    if (bh == by_holder_.end()) return freed;
    std::unordered_set<std::string> held;
    held.swap(bh->second);
    by_holder_.erase(bh);
    for (const std::string& o : held) {
      auto it = objs_.find(o);
      if (it == objs_.end()) continue;
      auto& hs = it->second.holders;
      for (size_t i = 0; i < hs.size(); ++i) {
        if (hs[i] == h) {
          hs[i] = hs.back();
          hs.pop_back();
          break;
        }
      }
      if (hs.empty() && it->second.pins <= 0) freed.emplace_back(o);
    }
    return freed;
  }

  std::vector<py::bytes> held_by(const std::string& key) const {
    std::vector<py::bytes> out;
    uint32_t h;
    if (!keys_.find(key, h)) return out;
    auto bh = by_holder_.find(h);
    if (bh != by_holder_.end())
      for (const std::string& o : bh->second) out.emplace_back(o);
    return out;
  }

  // Location of the value (node whose store holds it); "" clears it.
  void set_node(const py::bytes& oid, const std::string& node) {
    const std::string o(oid);
    Rec& r = objs_[o];
    if (r.node != kNoNode) unindex_node(r.node, o);
    r.node = node.empty() ? kNoNode : nodes_.id(node);
    if (r.node != kNoNode) by_node_[r.node].insert(o);
  }

  py::object node(const py::bytes& oid) const {
    auto it = objs_.find(std::string(oid));
    if (it == objs_.end() || it->second.node == kNoNode) return py::none();
    return py::str(nodes_.name(it->second.node));
  }

  std::vector<py::bytes> objects_on_node(const std::string& node) const {
    std::vector<py::bytes> out;
    uint32_t n;
    if (!nodes_.find(node, n)) return out;
    auto bn = by_node_.find(n);
    if (bn != by_node_.end())
      for (const std::string& o : bn->second) out.emplace_back(o);
    return out;
  }

  py::dict stats() const {
    size_t refs = 0, pinned = 0;
    for (const auto& kv : objs_) {
      refs += kv.second.holders.size();
      pinned += kv.second.pins > 0;
    }
    py::dict d;
    d["objects"] = objs_.size();
    d["holder_refs"] = refs;
    d["pinned_objects"] = pinned;
    d["holders"] = by_holder_.size();
    return d;
  }

 private:
  void unindex_holder(uint32_t h, const std::string& o) {
    auto bh = by_holder_.find(h);
    if (bh == by_holder_.end()) return;
    bh->second.erase(o);
    if (bh->second.empty()) by_holder_.erase(bh);
  }
  void unindex_node(uint32_t n, const std::string& o) {
    auto bn = by_node_.find(n);
    if (bn == by_node_.end()) return;
    bn->second.erase(o);
    if (bn->second.empty()) by_node_.erase(bn);
  }

  std::unordered_map<std::string, Rec> objs_;
  Interner keys_, nodes_;
  std::unordered_map<uint32_t, std::unordered_set<std::string>> by_holder_;
  std::unordered_map<uint32_t, std::unordered_set<std::string>> by_node_;
};

}  // namespace

void register_ref_table(py::module_& m) {
  py::class_<RefTable>(m, "RefTable")
      .def(py::init<>())
      .def("add", &RefTable::add)
      .def("contains", &RefTable::contains)
      .def("__len__", &RefTable::size)
      .def("erase", &RefTable::erase)
      .def("add_holder", &RefTable::add_holder)
      .def("remove_holder", &RefTable::remove_holder)
      .def("has_holder", &RefTable::has_holder)
      .def("pin", &RefTable::pin, py::arg("oid"), py::arg("n") = 1)
      .def("pins", &RefTable::pins)
      .def("num_holders", &RefTable::num_holders)
      .def("holders", &RefTable::holders)
      .def("referenced", &RefTable::referenced)
      .def("unreferenced", &RefTable::unreferenced)
      .def("clear_refs", &RefTable::clear_refs)
      .def("drop_holder", &RefTable::drop_holder)
      .def("held_by", &RefTable::held_by)
      .def("set_node", &RefTable::set_node)
      .def("node", &RefTable::node)
      .def("objects_on_node", &RefTable::objects_on_node)
      .def("stats", &RefTable::stats);
}
