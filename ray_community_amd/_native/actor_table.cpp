// Actor directory of the control plane (reference: the GCS actor table and its indexes,
// src/ray/gcs/gcs_server/gcs_actor_manager.h -- registered_actors_, named_actors_,
// created_actors_ per node, owners_ -- and the placement-group -> actors relation the PG manager
// walks on removal).
//
// The head keeps each actor's runtime handles (call queue, in-flight calls, waiters) in Python;
// this table owns the state an actor is LOOKED UP by, with an index per question the head asks:
//   (namespace, name) -> actor         get_actor / name reservation (a DEAD holder frees the name)
//   node -> actors                     node death, per-node listings
//   placement group -> actors          remove_placement_group kills the group's actors
//   holder -> actors, actor -> holders handle reference counting; a dying process drops all its
//                                      handles in one call (drop_holder) instead of a scan
//   state -> count                     metrics / summaries without a scan
// Keys are bytes (str keys are tagged so "a" and b"a" stay distinct). Not thread-safe: the head
// calls it under its lock.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace {

std::string key_of(const py::handle& o) {
  if (py::isinstance<py::bytes>(o)) return std::string(py::reinterpret_borrow<py::bytes>(o));
  if (py::isinstance<py::str>(o)) return "\x01" + py::reinterpret_borrow<py::str>(o).cast<std::string>();
  if (o.is_none()) return std::string("\0", 1);
  return "\x02" + py::str(o).cast<std::string>();  // ints and other hashables: by their text
}

using Set = std::unordered_set<std::string>;

class ActorDirectory {
 public:
  explicit ActorDirectory(std::string dead_state) : dead_(std::move(dead_state)) {}

  // Registers an actor. A name already held by a live (not dead) actor raises ValueError.
  void add(const py::bytes& aid_b, const py::object& name, const std::string& ns, const py::object& owner,
           const py::object& pg, const std::string& state, const std::string& cls, bool detached) {
    const std::string aid = aid_b;
    if (recs_.count(aid)) throw py::value_error("actor already registered");
    std::string nm = name.is_none() ? std::string() : py::str(name).cast<std::string>();
    if (!nm.empty()) {
      auto it = names_.find({ns, nm});
      if (it != names_.end() && it->second != aid) {
        auto r = recs_.find(it->second);
        if (r != recs_.end() && r->second.state != dead_)
          throw py::value_error("The name " + nm + " (namespace=" + ns + ") is already taken.");
      }
      names_[{ns, nm}] = aid;
    }
    Rec& r = recs_[aid];
    r.state = state;
    r.name = nm;
    r.ns = ns;
    r.cls = cls;
    r.detached = detached;
    r.pg = pg.is_none() ? std::string() : key_of(pg);
    if (!r.pg.empty()) by_pg_[r.pg].insert(aid);
    counts_[state] += 1;
    if (!owner.is_none()) add_handle(aid_b, owner);
  }

  bool contains(const py::bytes& aid) const { return recs_.count(std::string(aid)) != 0; }

  void set_state(const py::bytes& aid_b, const std::string& state) {
    Rec* r = find(aid_b);
    if (r == nullptr || r->state == state) return;
    counts_[r->state] -= 1;
    counts_[state] += 1;
    r->state = state;
  }

  void set_node(const py::bytes& aid_b, const py::object& node) {
    const std::string aid = aid_b;
    Rec* r = find(aid_b);
    if (r == nullptr) return;
    if (!r->node.empty()) erase_from(by_node_, r->node, aid);
    r->node = node.is_none() ? std::string() : key_of(node);
    if (!r->node.empty()) by_node_[r->node].insert(aid);
  }

  // Handle references: returns the actor's holder count after the change.
  size_t add_handle(const py::bytes& aid_b, const py::object& holder) {
    const std::string aid = aid_b;
    Rec* r = find(aid_b);
    if (r == nullptr) return 0;
    const std::string h = key_of(holder);
    if (r->holders.insert(h).second) by_holder_[h].insert(aid);
    return r->holders.size();
  }

  size_t remove_handle(const py::bytes& aid_b, const py::object& holder) {
    const std::string aid = aid_b;
    Rec* r = find(aid_b);
    if (r == nullptr) return 0;
    const std::string h = key_of(holder);
    if (r->holders.erase(h)) erase_from(by_holder_, h, aid);
    return r->holders.size();
  }

  size_t num_handles(const py::bytes& aid_b) const {
    auto it = recs_.find(std::string(aid_b));
    return it == recs_.end() ? 0 : it->second.holders.size();
  }

  // Drops every handle ``holder`` has; returns the actors that lost one (for the unreferenced check).
  std::vector<py::bytes> drop_holder(const py::object& holder) {
    std::vector<py::bytes> out;
    const std::string h = key_of(holder);
    auto it = by_holder_.find(h);
    if (it == by_holder_.end()) return out;
    for (const auto& aid : it->second) {
      auto r = recs_.find(aid);
      if (r != recs_.end()) r->second.holders.erase(h);
      out.emplace_back(aid);
    }
    by_holder_.erase(it);
    return out;
  }

  py::object by_name(const std::string& ns, const std::string& name) const {
    auto it = names_.find({ns, name});
    if (it == names_.end()) return py::none();
    return py::bytes(it->second);
  }

  bool name_available(const std::string& ns, const std::string& name) const {
    auto it = names_.find({ns, name});
    if (it == names_.end()) return true;
    auto r = recs_.find(it->second);
    return r == recs_.end() || r->second.state == dead_;
  }

  std::vector<py::bytes> on_node(const py::object& node) const { return members(by_node_, key_of(node)); }
  std::vector<py::bytes> in_pg(const py::object& pg) const { return members(by_pg_, key_of(pg)); }

  std::vector<py::bytes> named(const std::string& ns, bool all_namespaces) const {
    std::vector<py::bytes> out;
    for (const auto& kv : names_) {
      if (!all_namespaces && kv.first.first != ns) continue;
      auto r = recs_.find(kv.second);
      if (r != recs_.end() && r->second.state != dead_) out.emplace_back(kv.second);
    }
    return out;
  }

  std::map<std::string, int64_t> state_counts() const {
    std::map<std::string, int64_t> out;
    for (const auto& kv : counts_)
      if (kv.second) out.emplace(kv.first, kv.second);
    return out;
  }

  // Forgets an actor entirely (its name is released when it still points here).
  void remove(const py::bytes& aid_b) {
    const std::string aid = aid_b;
    auto it = recs_.find(aid);
    if (it == recs_.end()) return;
    Rec& r = it->second;
    counts_[r.state] -= 1;
    if (!r.node.empty()) erase_from(by_node_, r.node, aid);
    if (!r.pg.empty()) erase_from(by_pg_, r.pg, aid);
    for (const auto& h : r.holders) erase_from(by_holder_, h, aid);
    if (!r.name.empty()) {
      auto n = names_.find({r.ns, r.name});
      if (n != names_.end() && n->second == aid) names_.erase(n);
    }
    recs_.erase(it);
  }

  size_t size() const { return recs_.size(); }

 private:
  struct Rec {
    std::string state, name, ns, node, pg, cls;
    bool detached = false;
    Set holders;
  };

  Rec* find(const py::bytes& aid) {
    auto it = recs_.find(std::string(aid));
    return it == recs_.end() ? nullptr : &it->second;
  }

  static void erase_from(std::unordered_map<std::string, Set>& idx, const std::string& k, const std::string& aid) {
    auto it = idx.find(k);
    if (it == idx.end()) return;
    it->second.erase(aid);
    if (it->second.empty()) idx.erase(it);
  }

  static std::vector<py::bytes> members(const std::unordered_map<std::string, Set>& idx, const std::string& k) {
    std::vector<py::bytes> out;
    auto it = idx.find(k);
    if (it != idx.end())
      for (const auto& a : it->second) out.emplace_back(a);
    return out;
  }

  std::string dead_;
  std::unordered_map<std::string, Rec> recs_;
  std::map<std::pair<std::string, std::string>, std::string> names_;
  std::unordered_map<std::string, Set> by_node_, by_pg_, by_holder_;
  std::unordered_map<std::string, int64_t> counts_;
};

}  // namespace

void register_actor_table(py::module_& m) {
  py::class_<ActorDirectory>(m, "ActorDirectory")
      .def(py::init<std::string>(), py::arg("dead_state"))
      .def("add", &ActorDirectory::add, py::arg("aid"), py::arg("name"), py::arg("namespace"), py::arg("owner"),
           py::arg("pg"), py::arg("state"), py::arg("class_name") = "", py::arg("detached") = false)
      .def("__contains__", &ActorDirectory::contains)
      .def("set_state", &ActorDirectory::set_state)
      .def("set_node", &ActorDirectory::set_node)
      .def("add_handle", &ActorDirectory::add_handle)
      .def("remove_handle", &ActorDirectory::remove_handle)
      .def("num_handles", &ActorDirectory::num_handles)
      .def("drop_holder", &ActorDirectory::drop_holder)
      .def("by_name", &ActorDirectory::by_name)
      .def("name_available", &ActorDirectory::name_available)
      .def("on_node", &ActorDirectory::on_node)
      .def("in_pg", &ActorDirectory::in_pg)
      .def("named", &ActorDirectory::named, py::arg("namespace") = "", py::arg("all_namespaces") = false)
      .def("state_counts", &ActorDirectory::state_counts)
      .def("remove", &ActorDirectory::remove)
      .def("__len__", &ActorDirectory::size);
}
