// Placement-group directory of the control plane (reference: the GCS placement-group table,
// src/ray/gcs/gcs_server/gcs_placement_group_manager.h -- registered_placement_groups_,
// named_placement_groups_, the pending queue the scheduler drains, and the per-state counts its
// debug string reports).
//
// Bundle placement itself is the native scheduler's (scheduler.cpp, create_pg / remove_pg); this
// table owns what a placement group is LOOKED UP by:
//   pg id -> record          state, name, strategy, bundles, bundle -> node assignment, lifetime
//   name -> pg id            get_placement_group(name) without a scan (a REMOVED group frees it)
//   pending FIFO             groups still waiting for resources, in creation order
//   state -> count           metrics / summaries without a scan
// The head keeps only the waiters (Python futures of pg.ready()) beside it. Not thread-safe: the
// head calls it under its lock.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace {

const char* kRemoved = "REMOVED";

std::string hex_of(const std::string& b) {
  static const char* d = "0123456789abcdef";
  std::string out;
  out.reserve(b.size() * 2);
  for (unsigned char c : b) {
    out.push_back(d[c >> 4]);
    out.push_back(d[c & 15]);
  }
  return out;
}

class PgDirectory {
 public:
  // Registers a PENDING group at the back of the pending queue. ``bundles``: list of resource dicts
  // (kept as given); ``infeasible``: some bundle fits no node at all.
  void add(const py::bytes& pg_b, const std::string& name, const std::string& strategy, const py::list& bundles,
           const py::object& lifetime, double created, bool infeasible) {
    const std::string pg = pg_b;
    if (recs_.count(pg)) throw py::value_error("placement group already registered");
    // a live group already holds the name: reject, as the GCS does (a second registration would
    // overwrite the index and orphan the first group's lookup once the newer one is removed)
    if (!name.empty() && !by_name(name).is_none())
      throw py::value_error("Failed to create placement group '" + name + "' because name already exists.");
    Rec& r = recs_[pg];
    r.name = name;
    r.strategy = strategy;
    r.bundles = bundles;
    r.lifetime = lifetime.is_none() ? std::string() : py::str(lifetime).cast<std::string>();
    r.created = created;
    r.infeasible = infeasible;
    r.state = "PENDING";
    counts_[r.state] += 1;
    if (!name.empty()) names_[name] = pg;
    pending_.push_back(pg);
  }

  bool contains(const py::bytes& pg) const { return recs_.count(std::string(pg)) != 0; }
  size_t size() const { return recs_.size(); }

  // "" for an unknown group
  std::string state(const py::bytes& pg) const {
    auto it = recs_.find(std::string(pg));
    return it == recs_.end() ? std::string() : it->second.state;
  }

  void set_state(const py::bytes& pg_b, const std::string& st) {
    Rec& r = get(pg_b);
    if (r.state == st) return;
    counts_[r.state] -= 1;
    counts_[st] += 1;
    r.state = st;
    if (st != "PENDING") drop_pending(pg_b);
  }

  void set_nodes(const py::bytes& pg_b, const std::vector<std::string>& nodes) {
    Rec& r = get(pg_b);
    r.nodes = nodes;
    r.placed = true;
  }

  py::object nodes(const py::bytes& pg_b) {
    const Rec& r = get(pg_b);
    if (!r.placed) return py::none();
    return py::cast(r.nodes);
  }

  py::list bundles(const py::bytes& pg_b) { return get(pg_b).bundles; }
  std::string strategy(const py::bytes& pg_b) { return get(pg_b).strategy; }
  bool infeasible(const py::bytes& pg_b) { return get(pg_b).infeasible; }

  // the id of the live (not REMOVED) group registered under ``name``, else None
  py::object by_name(const std::string& name) const {
    auto it = names_.find(name);
    if (it == names_.end()) return py::none();
    auto r = recs_.find(it->second);
    if (r == recs_.end() || r->second.state == kRemoved) return py::none();
    return py::bytes(it->second);
  }

  py::list pending() const {
    py::list out;
    for (const auto& pg : pending_) out.append(py::bytes(pg));
    return out;
  }

  void drop_pending(const py::bytes& pg_b) {
    const std::string pg = pg_b;
    auto it = std::find(pending_.begin(), pending_.end(), pg);
    if (it != pending_.end()) pending_.erase(it);
  }

  // rpc_pg_table's record format
  py::dict info(const py::bytes& pg_b) {
    const std::string pg = pg_b;
    auto it = recs_.find(pg);
    if (it == recs_.end()) return py::dict();
    return info_of(pg, it->second);
  }

  py::dict table() {
    py::dict out;
    for (const auto& kv : recs_) out[py::str(hex_of(kv.first))] = info_of(kv.first, kv.second);
    return out;
  }

  std::map<std::string, long> state_counts() const {
    std::map<std::string, long> out;
    for (const auto& kv : counts_)
      if (kv.second > 0) out[kv.first] = kv.second;
    return out;
  }

 private:
  struct Rec {
    std::string name, strategy, state, lifetime;
    py::list bundles;
    std::vector<std::string> nodes;
    bool placed = false, infeasible = false;
    double created = 0.0;
  };

  Rec& get(const py::bytes& pg_b) {
    auto it = recs_.find(std::string(pg_b));
    if (it == recs_.end()) throw py::key_error("unknown placement group");
    return it->second;
  }

  py::dict info_of(const std::string& pg, const Rec& r) {
    py::dict b, n;
    for (size_t i = 0; i < r.bundles.size(); ++i) b[py::int_(i)] = py::dict(r.bundles[i]);
    for (size_t i = 0; i < r.nodes.size(); ++i) n[py::int_(i)] = py::str(r.nodes[i]);
    py::dict d;
    d["placement_group_id"] = hex_of(pg);
    d["name"] = r.name;
    d["strategy"] = r.strategy;
    d["state"] = r.state;
    d["bundles"] = b;
    d["bundles_to_node_id"] = n;
    return d;
  }

  std::unordered_map<std::string, Rec> recs_;
  std::unordered_map<std::string, std::string> names_;
  std::deque<std::string> pending_;
  std::map<std::string, long> counts_;
};

}  // namespace

void register_pg_table(py::module_& m) {
  py::class_<PgDirectory>(m, "PgDirectory")
      .def(py::init<>())
      .def("add", &PgDirectory::add, py::arg("pg_id"), py::arg("name"), py::arg("strategy"), py::arg("bundles"),
           py::arg("lifetime"), py::arg("created"), py::arg("infeasible"))
      .def("state", &PgDirectory::state)
      .def("set_state", &PgDirectory::set_state)
      .def("set_nodes", &PgDirectory::set_nodes)
      .def("nodes", &PgDirectory::nodes)
      .def("bundles", &PgDirectory::bundles)
      .def("strategy", &PgDirectory::strategy)
      .def("infeasible", &PgDirectory::infeasible)
      .def("by_name", &PgDirectory::by_name)
      .def("pending", &PgDirectory::pending)
      .def("drop_pending", &PgDirectory::drop_pending)
      .def("info", &PgDirectory::info)
      .def("table", &PgDirectory::table)
      .def("state_counts", &PgDirectory::state_counts)
      .def("__contains__", &PgDirectory::contains)
      .def("__len__", &PgDirectory::size);
}
