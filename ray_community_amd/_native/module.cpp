// _rca_native: C++ runtime core (shared-memory object store, cluster resource scheduler, I/O reactor,
// object reference table, internal KV, actor directory, placement-group directory,
// worker-pool index).
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_store(py::module_& m);
void register_scheduler(py::module_& m);
void register_reactor(py::module_& m);
void register_ref_table(py::module_& m);
void register_kv_table(py::module_& m);
void register_actor_table(py::module_& m);
void register_pg_table(py::module_& m);
void register_worker_pool(py::module_& m);

PYBIND11_MODULE(_rca_native, m) {
  m.doc() = "ray_community_amd native runtime core";
  register_store(m);
  register_scheduler(m);
  register_reactor(m);
  register_ref_table(m);
  register_kv_table(m);
  register_actor_table(m);
  register_pg_table(m);
  register_worker_pool(m);
}
