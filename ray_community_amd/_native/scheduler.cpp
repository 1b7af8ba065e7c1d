// Cluster resource scheduler (reference: src/ray/raylet/scheduling/{cluster_resource_scheduler,
// policy/hybrid_scheduling_policy,policy/spread_scheduling_policy}.cc and
// src/ray/gcs/gcs_server/gcs_placement_group_scheduler.cc).
//
// * Resources are interned to dense ids and stored as fixed-point int64 (1e-4 units), so
//   fractional GPUs/CPUs are exact.
// * Pending work is kept per *scheduling class* (same demand + strategy): FIFO inside a class,
//   classes are visited round-robin so a blocked class never starves others (head-of-line
//   blocking only within one class — the same property Ray's ClusterTaskManager has).
// * Policies: DEFAULT = hybrid (prefer the submitter's node while its critical-resource
//   utilisation stays below `spread_threshold`, else the least-utilised feasible node),
//   SPREAD = round-robin over feasible nodes, NODE_AFFINITY (hard/soft).
// * Placement groups reserve bundles atomically (PACK / SPREAD / STRICT_PACK / STRICT_SPREAD)
//   and expose them as renamed resources `<R>_group_<i>_<pg>` and `<R>_group_<pg>` (+ the
//   `bundle` resource), exactly the indirection Ray uses, so PG tasks schedule through the
//   ordinary resource path.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

static constexpr double kUnit = 10000.0;
static inline int64_t fx(double v) { return (int64_t)std::llround(v * kUnit); }
static inline double unfx(int64_t v) { return (double)v / kUnit; }

enum Strategy : int { DEFAULT = 0, SPREAD = 1, NODE_AFFINITY = 2 };

struct Demand {
  std::vector<std::pair<int, int64_t>> items;  // (resource id, amount)
};

struct NodeRec {
  std::string id;
  std::vector<int64_t> total, avail;
  bool alive = true;
};

struct PendingItem {
  int64_t key;
  std::string preferred;
  std::string affinity_node;
  bool affinity_soft = false;
};

struct SchedClass {
  Demand demand;
  int strategy;
  std::deque<PendingItem> q;
};

struct PGRec {
  std::string id;
  std::vector<std::map<std::string, double>> bundles;
  std::vector<std::string> nodes;  // node per bundle
};

class Scheduler {
 public:
  explicit Scheduler(double spread_threshold = 0.5) : spread_threshold_(spread_threshold) {}

  int rid(const std::string& name) {
    auto it = rid_.find(name);
    if (it != rid_.end()) return it->second;
    int id = (int)rnames_.size();
    rid_[name] = id;
    rnames_.push_back(name);
    for (auto& n : nodes_) {
      n.total.push_back(0);
      n.avail.push_back(0);
    }
    return id;
  }

  void add_node(const std::string& node_id, const std::map<std::string, double>& res) {
    if (node_index_.count(node_id)) throw std::runtime_error("node exists: " + node_id);
    for (auto& kv : res) rid(kv.first);
    NodeRec n;
    n.id = node_id;
    n.total.assign(rnames_.size(), 0);
    n.avail.assign(rnames_.size(), 0);
    for (auto& kv : res) {
      n.total[rid_[kv.first]] = fx(kv.second);
      n.avail[rid_[kv.first]] = fx(kv.second);
    }
    node_index_[node_id] = (int)nodes_.size();
    nodes_.push_back(n);
  }

  void remove_node(const std::string& node_id) {
    auto it = node_index_.find(node_id);
    if (it == node_index_.end()) return;
    NodeRec& n = nodes_[it->second];
    n.alive = false;
    std::fill(n.avail.begin(), n.avail.end(), 0);
    std::fill(n.total.begin(), n.total.end(), 0);
  }

  // add (delta > 0) or remove (delta < 0) resource capacity on a node (total and available)
  void adjust(const std::string& node_id, const std::map<std::string, double>& delta) {
    NodeRec& n = node(node_id);
    for (auto& kv : delta) {
      int r = rid(kv.first);
      n.total[r] += fx(kv.second);
      n.avail[r] += fx(kv.second);
      if (n.total[r] <= 0) {
        n.total[r] = 0;
        n.avail[r] = 0;
      }
    }
  }

  Demand make_demand(const std::map<std::string, double>& d) {
    Demand out;
    for (auto& kv : d) {
      if (kv.second <= 0) continue;
      out.items.push_back({rid(kv.first), fx(kv.second)});
    }
    std::sort(out.items.begin(), out.items.end());
    return out;
  }

  bool fits_avail(const NodeRec& n, const Demand& d) const {
    if (!n.alive) return false;
    for (auto& it : d.items)
      if (n.avail[it.first] < it.second) return false;
    return true;
  }
  bool fits_total(const NodeRec& n, const Demand& d) const {
    if (!n.alive) return false;
    for (auto& it : d.items)
      if (n.total[it.first] < it.second) return false;
    return true;
  }

  // critical-resource utilisation after placing d (hybrid policy score)
  double score(const NodeRec& n, const Demand& d) const {
    double s = 0.0;
    for (auto& it : d.items) {
      int64_t tot = n.total[it.first];
      if (tot <= 0) continue;
      double u = (double)(tot - n.avail[it.first] + it.second) / (double)tot;
      s = std::max(s, u);
    }
    return s;
  }

  bool feasible_anywhere(const Demand& d) const {
    for (auto& n : nodes_)
      if (fits_total(n, d)) return true;
    return false;
  }

  // choose a node with available resources now; "" if none
  std::string pick(const Demand& d, int strategy, const std::string& preferred, const std::string& affinity,
                   bool soft) {
    if (strategy == NODE_AFFINITY) {
      auto it = node_index_.find(affinity);
      if (it != node_index_.end() && fits_avail(nodes_[it->second], d)) return affinity;
      if (it != node_index_.end() && nodes_[it->second].alive && fits_total(nodes_[it->second], d) && !soft) return "";
      if (!soft) return "";
      strategy = DEFAULT;
    }
    if (strategy == SPREAD) {
      const int N = (int)nodes_.size();
      for (int k = 0; k < N; ++k) {
        int i = (spread_rr_ + k) % N;
        if (fits_avail(nodes_[i], d)) {
          spread_rr_ = (i + 1) % N;
          return nodes_[i].id;
        }
      }
      return "";
    }
    // hybrid
    if (!preferred.empty()) {
      auto it = node_index_.find(preferred);
      if (it != node_index_.end()) {
        const NodeRec& n = nodes_[it->second];
        if (fits_avail(n, d) && score(n, d) <= spread_threshold_) return n.id;
      }
    }
    int best = -1;
    double bs = 1e30;
    for (int i = 0; i < (int)nodes_.size(); ++i) {
      const NodeRec& n = nodes_[i];
      if (!fits_avail(n, d)) continue;
      double s = score(n, d);
      if (!preferred.empty() && n.id == preferred) s -= 1e-9;  // tie-break towards locality
      if (s < bs) {
        bs = s;
        best = i;
      }
    }
    return best < 0 ? std::string() : nodes_[best].id;
  }

  void acquire_d(const std::string& node_id, const Demand& d) {
    NodeRec& n = node(node_id);
    for (auto& it : d.items) n.avail[it.first] -= it.second;
  }
  void release_d(const std::string& node_id, const Demand& d) {
    NodeRec& n = node(node_id);
    if (!n.alive) return;
    for (auto& it : d.items) n.avail[it.first] = std::min(n.total[it.first], n.avail[it.first] + it.second);
  }

  // ------------------------------------------------------------------ python API
  py::object try_acquire(const std::map<std::string, double>& demand, int strategy, const std::string& preferred,
                         const std::string& affinity, bool soft) {
    Demand d = make_demand(demand);
    std::string n = pick(d, strategy, preferred, affinity, soft);
    if (n.empty()) return py::none();
    acquire_d(n, d);
    return py::str(n);
  }

  bool acquire(const std::string& node_id, const std::map<std::string, double>& demand, bool force) {
    Demand d = make_demand(demand);
    NodeRec& n = node(node_id);
    if (!force && !fits_avail(n, d)) return false;
    acquire_d(node_id, d);
    return true;
  }

  void release(const std::string& node_id, const std::map<std::string, double>& demand) {
    if (!node_index_.count(node_id)) return;
    release_d(node_id, make_demand(demand));
  }

  bool is_feasible(const std::map<std::string, double>& demand) { return feasible_anywhere(make_demand(demand)); }

  void enqueue(int64_t key, const std::map<std::string, double>& demand, int strategy, const std::string& preferred,
               const std::string& affinity, bool soft) {
    Demand d = make_demand(demand);
    std::string sig = std::to_string(strategy) + "|";
    for (auto& it : d.items) sig += std::to_string(it.first) + ":" + std::to_string(it.second) + ",";
    auto itc = class_index_.find(sig);
    int ci;
    if (itc == class_index_.end()) {
      ci = (int)classes_.size();
      class_index_[sig] = ci;
      classes_.push_back(SchedClass{d, strategy, {}});
    } else {
      ci = itc->second;
    }
    classes_[ci].q.push_back(PendingItem{key, preferred, affinity, soft});
    key_class_[key] = ci;
    ++num_pending_;
  }

  bool cancel(int64_t key) {
    auto it = key_class_.find(key);
    if (it == key_class_.end()) return false;
    auto& q = classes_[it->second].q;
    for (auto qi = q.begin(); qi != q.end(); ++qi) {
      if (qi->key == key) {
        q.erase(qi);
        key_class_.erase(it);
        --num_pending_;
        return true;
      }
    }
    return false;
  }

  // grant as much pending work as fits; returns [(key, node_id)] with resources acquired
  std::vector<std::pair<int64_t, std::string>> schedule(int max_grants) {
    std::vector<std::pair<int64_t, std::string>> out;
    if (num_pending_ == 0) return out;
    const int C = (int)classes_.size();
    bool progress = true;
    while (progress && (max_grants <= 0 || (int)out.size() < max_grants)) {
      progress = false;
      for (int k = 0; k < C; ++k) {
        SchedClass& c = classes_[(rr_ + k) % C];
        if (c.q.empty()) continue;
        PendingItem& p = c.q.front();
        std::string n = pick(c.demand, c.strategy, p.preferred, p.affinity_node, p.affinity_soft);
        if (n.empty()) continue;
        acquire_d(n, c.demand);
        out.push_back({p.key, n});
        key_class_.erase(p.key);
        c.q.pop_front();
        --num_pending_;
        progress = true;
        if (max_grants > 0 && (int)out.size() >= max_grants) break;
      }
      rr_ = C ? (rr_ + 1) % C : 0;
    }
    return out;
  }

  // pending keys whose demand no alive node can ever satisfy
  std::vector<int64_t> infeasible() {
    std::vector<int64_t> out;
    for (auto& c : classes_) {
      if (c.q.empty() || feasible_anywhere(c.demand)) continue;
      for (auto& p : c.q) out.push_back(p.key);
    }
    return out;
  }

  int num_pending() const { return num_pending_; }

  // ------------------------------------------------------------------ placement groups
  // returns node ids per bundle (resources reserved) or None if it cannot be placed now
  py::object create_pg(const std::string& pg_id, const std::vector<std::map<std::string, double>>& bundles,
                       const std::string& strategy) {
    std::vector<Demand> ds;
    for (auto& b : bundles) ds.push_back(make_demand(b));
    // snapshot availability to place tentatively
    std::vector<std::vector<int64_t>> avail;
    for (auto& n : nodes_) avail.push_back(n.avail);
    auto fits = [&](int ni, const Demand& d) {
      if (!nodes_[ni].alive) return false;
      for (auto& it : d.items)
        if (avail[ni][it.first] < it.second) return false;
      return true;
    };
    auto take = [&](int ni, const Demand& d) {
      for (auto& it : d.items) avail[ni][it.first] -= it.second;
    };
    const int N = (int)nodes_.size();
    std::vector<int> place(ds.size(), -1);
    if (strategy == "STRICT_PACK") {
      for (int ni = 0; ni < N; ++ni) {
        auto saved = avail[ni];
        bool ok = true;
        for (auto& d : ds) {
          if (!fits(ni, d)) {
            ok = false;
            break;
          }
          take(ni, d);
        }
        if (ok) {
          std::fill(place.begin(), place.end(), ni);
          break;
        }
        avail[ni] = saved;
      }
    } else if (strategy == "STRICT_SPREAD") {
      std::vector<bool> used(N, false);
      for (size_t b = 0; b < ds.size(); ++b) {
        for (int ni = 0; ni < N; ++ni) {
          if (used[ni] || !fits(ni, ds[b])) continue;
          take(ni, ds[b]);
          used[ni] = true;
          place[b] = ni;
          break;
        }
      }
    } else if (strategy == "SPREAD") {
      int start = 0;
      for (size_t b = 0; b < ds.size(); ++b) {
        for (int k = 0; k < N; ++k) {
          int ni = (start + k) % N;
          if (!fits(ni, ds[b])) continue;
          take(ni, ds[b]);
          place[b] = ni;
          start = ni + 1;
          break;
        }
      }
    } else {  // PACK: as few nodes as possible, greedy on the node with most room
      for (size_t b = 0; b < ds.size(); ++b) {
        int prev = b > 0 ? place[b - 1] : -1;
        if (prev >= 0 && fits(prev, ds[b])) {
          take(prev, ds[b]);
          place[b] = prev;
          continue;
        }
        for (int ni = 0; ni < N; ++ni) {
          if (!fits(ni, ds[b])) continue;
          take(ni, ds[b]);
          place[b] = ni;
          break;
        }
      }
    }
    for (int p : place)
      if (p < 0) return py::none();
    // commit: subtract bundle resources, add renamed resources
    PGRec rec;
    rec.id = pg_id;
    rec.bundles = bundles;
    py::list nodes_out;
    for (size_t b = 0; b < ds.size(); ++b) {
      NodeRec& n = nodes_[place[b]];
      acquire_d(n.id, ds[b]);
      std::map<std::string, double> virt;
      for (auto& kv : bundles[b]) {
        if (kv.second <= 0) continue;
        virt[kv.first + "_group_" + std::to_string(b) + "_" + pg_id] += kv.second;
        virt[kv.first + "_group_" + pg_id] += kv.second;
      }
      virt["bundle_group_" + std::to_string(b) + "_" + pg_id] += 1000.0;
      virt["bundle_group_" + pg_id] += 1000.0;
      adjust(n.id, virt);
      rec.nodes.push_back(n.id);
      nodes_out.append(n.id);
    }
    pgs_[pg_id] = rec;
    return nodes_out;
  }

  bool remove_pg(const std::string& pg_id) {
    auto it = pgs_.find(pg_id);
    if (it == pgs_.end()) return false;
    PGRec& rec = it->second;
    for (size_t b = 0; b < rec.bundles.size(); ++b) {
      auto ni = node_index_.find(rec.nodes[b]);
      if (ni == node_index_.end()) continue;
      NodeRec& n = nodes_[ni->second];
      // drop renamed resources
      for (auto& kv : rec.bundles[b]) {
        if (kv.second <= 0) continue;
        for (std::string nm : {kv.first + "_group_" + std::to_string(b) + "_" + pg_id, kv.first + "_group_" + pg_id}) {
          int r = rid(nm);
          n.total[r] = 0;
          n.avail[r] = 0;
        }
      }
      for (std::string nm : {std::string("bundle_group_") + std::to_string(b) + "_" + pg_id, "bundle_group_" + pg_id}) {
        int r = rid(nm);
        n.total[r] = 0;
        n.avail[r] = 0;
      }
      release_d(n.id, make_demand(rec.bundles[b]));
    }
    pgs_.erase(it);
    return true;
  }

  std::map<std::string, std::map<std::string, double>> totals() const { return snapshot(true); }
  std::map<std::string, std::map<std::string, double>> available() const { return snapshot(false); }

  std::vector<std::string> node_ids() const {
    std::vector<std::string> out;
    for (auto& n : nodes_)
      if (n.alive) out.push_back(n.id);
    return out;
  }

 private:
  NodeRec& node(const std::string& id) {
    auto it = node_index_.find(id);
    if (it == node_index_.end()) throw std::runtime_error("unknown node " + id);
    return nodes_[it->second];
  }
  std::map<std::string, std::map<std::string, double>> snapshot(bool total) const {
    std::map<std::string, std::map<std::string, double>> out;
    for (auto& n : nodes_) {
      if (!n.alive) continue;
      auto& m = out[n.id];
      for (size_t r = 0; r < rnames_.size(); ++r) {
        int64_t v = total ? n.total[r] : n.avail[r];
        if (n.total[r] > 0) m[rnames_[r]] = unfx(v);
      }
    }
    return out;
  }

  double spread_threshold_;
  std::unordered_map<std::string, int> rid_;
  std::vector<std::string> rnames_;
  std::vector<NodeRec> nodes_;
  std::unordered_map<std::string, int> node_index_;
  std::vector<SchedClass> classes_;
  std::unordered_map<std::string, int> class_index_;
  std::unordered_map<int64_t, int> key_class_;
  std::map<std::string, PGRec> pgs_;
  int num_pending_ = 0;
  int rr_ = 0;
  int spread_rr_ = 0;
};

void register_scheduler(py::module_& m) {
  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<double>(), py::arg("spread_threshold") = 0.5)
      .def("add_node", &Scheduler::add_node)
      .def("remove_node", &Scheduler::remove_node)
      .def("adjust", &Scheduler::adjust)
      .def("try_acquire", &Scheduler::try_acquire, py::arg("demand"), py::arg("strategy") = 0,
           py::arg("preferred") = "", py::arg("affinity") = "", py::arg("soft") = false)
      .def("acquire", &Scheduler::acquire, py::arg("node_id"), py::arg("demand"), py::arg("force") = false)
      .def("release", &Scheduler::release)
      .def("is_feasible", &Scheduler::is_feasible)
      .def("enqueue", &Scheduler::enqueue, py::arg("key"), py::arg("demand"), py::arg("strategy") = 0,
           py::arg("preferred") = "", py::arg("affinity") = "", py::arg("soft") = false)
      .def("cancel", &Scheduler::cancel)
      .def("schedule", &Scheduler::schedule, py::arg("max_grants") = 0)
      .def("infeasible", &Scheduler::infeasible)
      .def("num_pending", &Scheduler::num_pending)
      .def("create_pg", &Scheduler::create_pg)
      .def("remove_pg", &Scheduler::remove_pg)
      .def("totals", &Scheduler::totals)
      .def("available", &Scheduler::available)
      .def("node_ids", &Scheduler::node_ids);
}
