// Worker-pool index of the node manager (reference: src/ray/raylet/worker_pool.h -- the per-language
// idle worker stacks PopWorker/PushWorker serve, the "starting" counts that keep PopWorker from
// over-spawning, and TryKillingIdleWorkers' soft limit + idle timeout, oldest idle first).
//
// The head keeps the worker processes themselves (WorkerState: socket, Popen, GPU objects); this
// index owns which of them are reusable and for what:
//   (node, env key) -> idle stack   LIFO, so the most recently used (warm) worker is reused first
//   worker -> (node, key, since)     O(1) removal when an idle worker dies or is retired
//   (node, env key) -> starting      processes spawned but not yet registered
// An env key is the head's (runtime_env json, assigned GPU ids) pair flattened to one string. Not
// thread-safe: the head calls it under its lock.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace {

class WorkerPool {
 public:
  // ``wid`` becomes reusable for tasks of ``key`` on ``node``; re-pushing an idle worker moves it
  void push_idle(const std::string& node, const std::string& key, const py::bytes& wid_b, double since) {
    const std::string wid = wid_b;
    remove(wid_b);
    stacks_[{node, key}].push_back(wid);
    idle_[wid] = Idle{node, key, since};
    idle_per_node_[node] += 1;
  }

  // the most recently pushed idle worker for (node, key), removed from the pool; None if none
  py::object pop_idle(const std::string& node, const std::string& key) {
    auto it = stacks_.find({node, key});
    if (it == stacks_.end() || it->second.empty()) return py::none();
    std::string wid = it->second.back();
    it->second.pop_back();
    if (it->second.empty()) stacks_.erase(it);
    idle_.erase(wid);
    idle_per_node_[node] -= 1;
    return py::bytes(wid);
  }

  // drops ``wid`` from the idle pool (it died, got an actor, or is being retired); True if it was idle
  bool remove(const py::bytes& wid_b) {
    const std::string wid = wid_b;
    auto it = idle_.find(wid);
    if (it == idle_.end()) return false;
    auto st = stacks_.find({it->second.node, it->second.key});
    if (st != stacks_.end()) {
      auto& v = st->second;
      v.erase(std::remove(v.begin(), v.end(), wid), v.end());
      if (v.empty()) stacks_.erase(st);
    }
    idle_per_node_[it->second.node] -= 1;
    idle_.erase(it);
    return true;
  }

  bool is_idle(const py::bytes& wid) const { return idle_.count(std::string(wid)) != 0; }

  // adjusts the spawned-not-registered count (never below zero) and returns the new value
  long add_starting(const std::string& node, const std::string& key, long delta) {
    long& n = starting_[{node, key}];
    n = std::max(0L, n + delta);
    return n;
  }

  long starting(const std::string& node, const std::string& key) const {
    auto it = starting_.find({node, key});
    return it == starting_.end() ? 0 : it->second;
  }

  long idle_count(const std::string& node) const {
    auto it = idle_per_node_.find(node);
    return it == idle_per_node_.end() ? 0 : it->second;
  }

  // TryKillingIdleWorkers: while ``node`` holds more than ``keep`` idle workers, remove those idle for
  // longer than ``timeout_s``, oldest first; returns the removed ids for the head to terminate
  std::vector<py::bytes> reap(const std::string& node, long keep, double timeout_s, double now) {
    std::vector<py::bytes> out;
    long n = idle_count(node);
    if (n <= keep) return out;
    std::vector<std::pair<double, std::string>> old;
    for (const auto& kv : idle_)
      if (kv.second.node == node && now - kv.second.since > timeout_s) old.emplace_back(kv.second.since, kv.first);
    std::sort(old.begin(), old.end());
    for (const auto& o : old) {
      if (n <= keep) break;
      remove(py::bytes(o.second));
      out.emplace_back(o.second);
      --n;
    }
    return out;
  }

  // a node left the cluster: forget its idle stacks and starting counts; returns its idle workers
  std::vector<py::bytes> drop_node(const std::string& node) {
    std::vector<py::bytes> out;
    for (auto it = idle_.begin(); it != idle_.end();) {
      if (it->second.node == node) {
        out.emplace_back(it->first);
        it = idle_.erase(it);
      } else {
        ++it;
      }
    }
    for (auto it = stacks_.begin(); it != stacks_.end();)
      it = it->first.first == node ? stacks_.erase(it) : std::next(it);
    for (auto it = starting_.begin(); it != starting_.end();)
      it = it->first.first == node ? starting_.erase(it) : std::next(it);
    idle_per_node_.erase(node);
    return out;
  }

  // {node: {"idle": n, "starting": m}} for metrics and the state API
  py::dict stats() const {
    py::dict out;
    auto row = [&](const std::string& node) -> py::dict {
      py::str k(node);
      if (!out.contains(k)) {
        py::dict d;
        d["idle"] = 0;
        d["starting"] = 0;
        out[k] = d;
      }
      return out[k].cast<py::dict>();
    };
    for (const auto& kv : idle_per_node_)
      if (kv.second > 0) row(kv.first)["idle"] = kv.second;
    std::map<std::string, long> st;
    for (const auto& kv : starting_) st[kv.first.first] += kv.second;
    for (const auto& kv : st)
      if (kv.second > 0) row(kv.first)["starting"] = kv.second;
    return out;
  }

  size_t size() const { return idle_.size(); }

 private:
  struct Idle {
    std::string node, key;
    double since;
  };
  std::map<std::pair<std::string, std::string>, std::vector<std::string>> stacks_;
  std::unordered_map<std::string, Idle> idle_;
  std::map<std::pair<std::string, std::string>, long> starting_;
  std::unordered_map<std::string, long> idle_per_node_;
};

}  // namespace

void register_worker_pool(py::module_& m) {
  py::class_<WorkerPool>(m, "WorkerPool")
      .def(py::init<>())
      .def("push_idle", &WorkerPool::push_idle, py::arg("node"), py::arg("key"), py::arg("wid"), py::arg("since"))
      .def("pop_idle", &WorkerPool::pop_idle)
      .def("remove", &WorkerPool::remove)
      .def("is_idle", &WorkerPool::is_idle)
      .def("add_starting", &WorkerPool::add_starting)
      .def("starting", &WorkerPool::starting)
      .def("idle_count", &WorkerPool::idle_count)
      .def("reap", &WorkerPool::reap, py::arg("node"), py::arg("keep"), py::arg("timeout_s"), py::arg("now"))
      .def("drop_node", &WorkerPool::drop_node)
      .def("stats", &WorkerPool::stats)
      .def("__len__", &WorkerPool::size);
}
