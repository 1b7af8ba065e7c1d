"""(reference: ``python/ray/util/joblib/ray_backend.py``)"""
from __future__ import annotations

from joblib._parallel_backends import MultiprocessingBackend

from ..multiprocessing import Pool


class RayBackend(MultiprocessingBackend):
    supports_timeout = True

    def effective_n_jobs(self, n_jobs):
        from ..._private import worker as w

        if not w.is_initialized():
            w.init()
        cpus = int(w.cluster_resources().get("CPU", 1))
        if n_jobs is None or n_jobs < 0:
            return max(1, cpus)
        return max(1, min(int(n_jobs), cpus * 4))

    def configure(self, n_jobs=1, parallel=None, prefer=None, require=None, **kwargs):
        n_jobs = self.effective_n_jobs(n_jobs)
        self._pool = Pool(processes=n_jobs)
        self.parallel = parallel
        return n_jobs

    def terminate(self):
        if getattr(self, "_pool", None) is not None:
            self._pool.terminate()
            self._pool = None
