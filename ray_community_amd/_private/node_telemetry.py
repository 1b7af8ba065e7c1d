"""Node and MI355X GPU telemetry for the dashboard's ``/metrics`` (reference:
``python/ray/dashboard/modules/reporter/reporter_agent.py`` METRICS_GAUGES and its GPU probes,
which read NVML / ``amdsmi``).

Sources, cheapest first, none of which initialises HIP in the reporting process:

  * AMD GPU sysfs (``/sys/class/drm/cardN/device``): ``mem_info_vram_used`` / ``_total`` (HBM
    bytes), ``gpu_busy_percent``, ``pp_dpm_sclk`` (current shader clock), hwmon ``power1_average``
    / ``power1_input`` (uW) and ``temp*_input`` (m degC, labelled edge / junction / mem);
  * ``amd-smi metric --json`` (``parse_amd_smi_metric``) when sysfs is not readable, e.g. inside
    containers that hide it; its JSON layout differs across ROCm releases (a bare list, or
    ``{"gpu_data": [...]}``; values as numbers, ``{"value", "unit"}`` dicts or "123 W" strings),
    so the parser normalises all of them;
  * ``psutil`` for node CPU / memory / disk.

Every GPU record has the same keys: index, name, vram_total / vram_used (bytes), busy_percent,
power_w, temp_c ({sensor: degC}), sclk_mhz (None where a source does not report a field).
Metric names follow the reference's (``ray_node_gpus_utilization``, ``ray_node_gram_used`` ...)
so existing Grafana dashboards keep working, plus MI355X extras (power, temperatures, clock).
"""
from __future__ import annotations

import glob
import json
import os
import re
import shutil
import subprocess
import time
from typing import Dict, List, Optional

_SYSFS_ROOT = "/sys/class/drm"
_CARD_RE = re.compile(r"card(\d+)$")


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _read_int(path: str) -> Optional[int]:
    s = _read(path)
    try:
        return int(s) if s is not None else None
    except ValueError:
        return None


def _current_sclk(text: Optional[str]) -> Optional[float]:
    """``pp_dpm_sclk``: lines like ``1: 2100Mhz *``; the starred one is the current level."""
    if not text:
        return None
    for ln in text.splitlines():
        if ln.rstrip().endswith("*"):
            m = re.search(r"(\d+(?:\.\d+)?)\s*[Mm][Hh]z", ln)
            if m:
                return float(m.group(1))
    return None


def read_gpus_sysfs(root: str = _SYSFS_ROOT) -> List[Dict]:
    cards = []
    for p in glob.glob(os.path.join(root, "card*")):
        m = _CARD_RE.search(os.path.basename(p))
        if m and os.path.exists(os.path.join(p, "device", "mem_info_vram_total")):
            cards.append((int(m.group(1)), p))
    out = []
    for i, (_, p) in enumerate(sorted(cards)):
        d = os.path.join(p, "device")
        try:
            pci = os.path.basename(os.path.realpath(d))
        except OSError:
            pci = ""
        rec = {"index": i, "pci": pci, "unique_id": (_read(os.path.join(d, "unique_id")) or "").lower(),
               "name": _read(os.path.join(d, "product_name")) or "AMD Instinct GPU",
               "vram_total": _read_int(os.path.join(d, "mem_info_vram_total")),
               "vram_used": _read_int(os.path.join(d, "mem_info_vram_used")),
               "busy_percent": _read_int(os.path.join(d, "gpu_busy_percent")),
               "sclk_mhz": _current_sclk(_read(os.path.join(d, "pp_dpm_sclk"))),
               "power_w": None, "temp_c": {}}
        for h in sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*"))):
            pw = _read_int(os.path.join(h, "power1_average"))
            if pw is None:
                pw = _read_int(os.path.join(h, "power1_input"))
            if pw is not None and rec["power_w"] is None:
                rec["power_w"] = pw / 1e6
            for t in sorted(glob.glob(os.path.join(h, "temp*_input"))):
                v = _read_int(t)
                if v is None:
                    continue
                label = _read(t.replace("_input", "_label")) or os.path.basename(t).split("_")[0]
                rec["temp_c"][label] = v / 1000.0
        out.append(rec)
    return out


# ----------------------------------------------------------------------------- amd-smi
_UNIT_BYTES = {"b": 1, "kb": 1 << 10, "kib": 1 << 10, "mb": 1 << 20, "mib": 1 << 20, "gb": 1 << 30, "gib": 1 << 30}


def _val(x):
    """(number, unit) from 12, "12", "12 W", {"value": 12, "unit": "W"}; (None, None) for N/A."""
    if isinstance(x, dict):
        if "value" in x:
            v, u = _val(x["value"])
            return v, (x.get("unit") or u)
        return None, None
    if isinstance(x, (int, float)) and not isinstance(x, bool):
        return float(x), None
    if isinstance(x, str):
        m = re.match(r"\s*(-?\d+(?:\.\d+)?)\s*([A-Za-z%/]*)", x)
        if m:
            return float(m.group(1)), (m.group(2) or None)
    return None, None


def _bytes(x) -> Optional[int]:
    v, u = _val(x)
    if v is None:
        return None
    return int(v * _UNIT_BYTES.get((u or "mb").lower(), 1 << 20))  # amd-smi reports VRAM in MB


def _first(d: Dict, *keys):
    for k in keys:
        if isinstance(d, dict) and k in d and d[k] not in (None, "N/A"):
            return d[k]
    return None


def parse_amd_smi_metric(text: str) -> List[Dict]:
    data = json.loads(text)
    if isinstance(data, dict):
        data = data.get("gpu_data") or data.get("gpus") or [data]
    out = []
    for i, g in enumerate(data):
        if not isinstance(g, dict):
            continue
        usage = g.get("usage") or {}
        mem = g.get("mem_usage") or g.get("memory_usage") or {}
        power = g.get("power") or {}
        temp = g.get("temperature") or {}
        clock = g.get("clock") or {}
        busy, _ = _val(_first(usage, "gfx_activity", "gfx_usage", "gpu_use_percent"))
        pw, _ = _val(_first(power, "socket_power", "average_socket_power", "current_socket_power"))
        sclk = None
        gfx = _first(clock, "gfx_0", "gfx", "sclk")
        if isinstance(gfx, dict):
            sclk, _ = _val(_first(gfx, "clk", "current", "value") if "value" not in gfx else gfx)
        temps = {}
        for k, v in (temp.items() if isinstance(temp, dict) else []):
            tv, _ = _val(v)
            if tv is not None:
                temps[k] = tv
        idx = g.get("gpu", i)
        out.append({"index": int(idx) if isinstance(idx, (int, float, str)) and str(idx).isdigit() else i,
                    "name": str(g.get("asic", {}).get("market_name")) if isinstance(g.get("asic"), dict)
                    else "AMD Instinct GPU",
                    "vram_total": _bytes(_first(mem, "total_vram", "vram_total")),
                    "vram_used": _bytes(_first(mem, "used_vram", "vram_used")),
                    "busy_percent": busy, "power_w": pw, "temp_c": temps, "sclk_mhz": sclk})
    return out


def read_gpus_amd_smi(timeout: float = 10.0) -> List[Dict]:
    exe = shutil.which("amd-smi") or ("/opt/rocm/bin/amd-smi" if os.path.exists("/opt/rocm/bin/amd-smi") else None)
    if exe is None:
        return []
    try:
        r = subprocess.run([exe, "metric", "--json"], capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired):
        return []
    if r.returncode != 0 or not r.stdout.strip():
        return []
    try:
        return parse_amd_smi_metric(r.stdout)
    except (ValueError, TypeError, AttributeError):
        return []


def visible_gpu_serials(timeout: float = 20.0) -> Optional[List[str]]:
    """ASIC serials of the GPUs this process may use, in device order (``amd-smi static --asic``
    honours the visibility the container / HIP_VISIBLE_DEVICES imposes; sysfs lists every GPU of
    the host, other tenants' included). None when amd-smi is unavailable."""
    exe = shutil.which("amd-smi") or ("/opt/rocm/bin/amd-smi" if os.path.exists("/opt/rocm/bin/amd-smi") else None)
    if exe is None:
        return None
    try:
        r = subprocess.run([exe, "static", "--asic", "--json"], capture_output=True, text=True, timeout=timeout)
        data = json.loads(r.stdout) if r.returncode == 0 and r.stdout.strip() else None
    except (OSError, subprocess.TimeoutExpired, ValueError):
        return None
    if data is None:
        return None
    return parse_amd_smi_serials(data)


def parse_amd_smi_serials(data) -> List[str]:
    if isinstance(data, str):
        data = json.loads(data)
    if isinstance(data, dict):
        data = data.get("gpu_data") or [data]
    out = []
    for g in sorted((g for g in data if isinstance(g, dict)), key=lambda g: int(g.get("gpu", 0))):
        ser = str((g.get("asic") or {}).get("asic_serial", "")).lower()
        out.append(ser[2:] if ser.startswith("0x") else ser)
    return out


def read_gpus(allow_amd_smi: bool = True, serials: Optional[List[str]] = None) -> List[Dict]:
    """GPU records; with ``serials`` (visible_gpu_serials) only those GPUs, indexed in that order."""
    g = read_gpus_sysfs()
    if g and serials:
        by = {r.get("unique_id"): r for r in g}
        sel = [by[s] for s in serials if s in by]
        if sel:
            for i, r in enumerate(sel):
                r["index"] = i
            g = sel
    if not g and allow_amd_smi:
        g = read_gpus_amd_smi()
    return g


# ----------------------------------------------------------------------------- node
def read_node() -> Dict:
    out = {"cpu_percent": None, "cpu_count": os.cpu_count(), "mem_total": None, "mem_used": None,
           "mem_available": None, "shm_used": None, "disk_total": None, "disk_used": None}
    try:
        import psutil

        out["cpu_percent"] = psutil.cpu_percent(interval=None)
        vm = psutil.virtual_memory()
        out.update(mem_total=vm.total, mem_used=vm.total - vm.available, mem_available=vm.available)
        out["shm_used"] = getattr(vm, "shared", None)
        du = psutil.disk_usage("/tmp")
        out.update(disk_total=du.total, disk_used=du.used)
    except Exception:  # noqa - psutil missing / restricted /proc: report what is known
        pass
    return out


class TelemetryCache:
    """Latest readings, refreshed every ``period_s`` by a daemon thread (a Prometheus scrape must
    neither wait for nor fork ``amd-smi``). The first ``get`` reads sysfs + psutil synchronously."""

    def __init__(self, period_s: float = 2.0, allow_amd_smi: bool = True):
        import threading

        self.period_s = period_s
        self.allow_amd_smi = allow_amd_smi
        self._lock = threading.Lock()
        self._node: Dict = {}
        self._gpus: List[Dict] = []
        self._thread = None

    def _refresh(self, allow_amd_smi):
        if not hasattr(self, "_serials"):
            self._serials = None if os.environ.get("RCA_TELEMETRY_ALL_GPUS") == "1" else visible_gpu_serials()
        node, gpus = read_node(), read_gpus(allow_amd_smi, self._serials)
        if allow_amd_smi and not gpus:
            self._smi_misses = getattr(self, "_smi_misses", 0) + 1
            if self._smi_misses >= 2:  # no AMD GPU visible to either source: stop forking amd-smi
                self.allow_amd_smi = False
        with self._lock:
            self._node, self._gpus = node, gpus

    def _loop(self):
        while True:
            try:
                self._refresh(self.allow_amd_smi)
            except Exception:  # noqa - telemetry must never take the head down
                pass
            time.sleep(self.period_s)

    def get(self):
        if self._thread is None:
            import threading

            with self._lock:
                self._node = read_node()
            # the first GPU read (which resolves the visible GPUs through amd-smi) runs on the thread
            self._thread = threading.Thread(target=self._loop, daemon=True, name="rca-telemetry")
            self._thread.start()
        with self._lock:
            return dict(self._node), list(self._gpus)


def prometheus_lines(node: Dict, gpus: List[Dict], ip: str, session: str) -> List[str]:
    lines: List[str] = []

    def gauge(name, help_, samples):
        samples = [(t, v) for t, v in samples if v is not None]
        if not samples:
            return
        lines.append(f"# HELP {name} {help_}")
        lines.append(f"# TYPE {name} gauge")
        for tags, v in samples:
            t = ",".join(f'{k}="{val}"' for k, val in tags.items())
            lines.append(f"{name}{{{t}}} {v}")

    base = {"ip": ip, "SessionName": session}
    gauge("ray_node_cpu_utilization", "Total CPU usage on a ray node", [(base, node.get("cpu_percent"))])
    gauge("ray_node_cpu_count", "Total CPUs available on a ray node", [(base, node.get("cpu_count"))])
    gauge("ray_node_mem_used", "Memory usage on a ray node", [(base, node.get("mem_used"))])
    gauge("ray_node_mem_available", "Memory available on a ray node", [(base, node.get("mem_available"))])
    gauge("ray_node_mem_total", "Total memory on a ray node", [(base, node.get("mem_total"))])
    gauge("ray_node_mem_shared_bytes", "Total shared memory usage on a ray node", [(base, node.get("shm_used"))])
    gauge("ray_node_disk_usage", "Used disk space on a ray node", [(base, node.get("disk_used"))])
    gauge("ray_node_disk_free", "Free disk space on a ray node",
          [(base, (node["disk_total"] - node["disk_used"]) if node.get("disk_total") is not None else None)])
    gt = [({**base, "GpuIndex": str(g["index"]), "GpuDeviceName": g.get("name") or ""}, g) for g in gpus]
    gauge("ray_node_gpus_available", "Total GPUs available on a ray node", [(t, 1) for t, _ in gt])
    gauge("ray_node_gpus_utilization", "Total GPUs usage on a ray node", [(t, g.get("busy_percent")) for t, g in gt])
    gauge("ray_node_gram_used", "Total GPU RAM (HBM) usage on a ray node (bytes)",
          [(t, g.get("vram_used")) for t, g in gt])
    gauge("ray_node_gram_available", "Total GPU RAM (HBM) available on a ray node (bytes)",
          [(t, (g["vram_total"] - g["vram_used"]) if g.get("vram_total") is not None and g.get("vram_used") is not None
            else None) for t, g in gt])
    gauge("ray_node_gram_total", "GPU RAM (HBM) capacity (bytes)", [(t, g.get("vram_total")) for t, g in gt])
    gauge("ray_node_gpu_power_watts", "GPU socket power (W)", [(t, g.get("power_w")) for t, g in gt])
    gauge("ray_node_gpu_sclk_mhz", "Current GPU shader clock (MHz)", [(t, g.get("sclk_mhz")) for t, g in gt])
    gauge("ray_node_gpu_temperature_celsius", "GPU temperatures by sensor (degC)",
          [({**t, "sensor": s}, v) for t, g in gt for s, v in (g.get("temp_c") or {}).items()])
    return lines
