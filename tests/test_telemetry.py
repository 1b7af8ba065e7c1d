"""Node / MI355X telemetry in /metrics (reference: dashboard/modules/reporter/reporter_agent.py
METRICS_GAUGES; tests/test_metrics_agent.py). sysfs reader on a synthetic card tree, amd-smi JSON
parser on the layouts ROCm releases emit (plus the capture from a real MI355X box when present in
tests/fixtures), Prometheus lines, and the head's /metrics endpoint."""
import json
import os
import urllib.request

import pytest

from ray_community_amd._private import node_telemetry as nt

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def _w(p, s):
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(s)


def test_sysfs_reader(tmp_path):
    d = tmp_path / "card1" / "device"
    _w(str(d / "mem_info_vram_total"), "309220868096\n")
    _w(str(d / "mem_info_vram_used"), "4294967296\n")
    _w(str(d / "gpu_busy_percent"), "87\n")
    _w(str(d / "pp_dpm_sclk"), "0: 500Mhz\n1: 2100Mhz *\n2: 2400Mhz\n")
    _w(str(d / "product_name"), "AMD Instinct MI355X\n")
    _w(str(d / "hwmon" / "hwmon3" / "power1_average"), "612000000\n")
    _w(str(d / "hwmon" / "hwmon3" / "temp1_input"), "45000\n")
    _w(str(d / "hwmon" / "hwmon3" / "temp1_label"), "edge\n")
    _w(str(d / "hwmon" / "hwmon3" / "temp2_input"), "61000\n")
    _w(str(d / "hwmon" / "hwmon3" / "temp2_label"), "junction\n")
    _w(str(tmp_path / "card1-DP-1" / "status"), "disconnected")  # connector entries are not GPUs
    _w(str(tmp_path / "card0" / "device" / "vendor"), "0x1234")   # no VRAM files: not an AMD GPU
    g = nt.read_gpus_sysfs(str(tmp_path))
    assert len(g) == 1
    r = g[0]
    assert r["index"] == 0 and r["name"] == "AMD Instinct MI355X"
    assert r["vram_total"] == 309220868096 and r["vram_used"] == 4 << 30 and r["busy_percent"] == 87
    assert r["sclk_mhz"] == 2100.0 and r["power_w"] == pytest.approx(612.0)
    assert r["temp_c"] == {"edge": 45.0, "junction": 61.0}


_AMD_SMI_DICT_VALUES = [{
    "gpu": 0,
    "usage": {"gfx_activity": {"value": 93, "unit": "%"}, "umc_activity": {"value": 40, "unit": "%"}},
    "power": {"socket_power": {"value": 987, "unit": "W"}},
    "clock": {"gfx_0": {"clk": {"value": 2085, "unit": "MHz"}}},
    "temperature": {"edge": {"value": 50, "unit": "C"}, "hotspot": {"value": 72, "unit": "C"},
                    "mem": {"value": 60, "unit": "C"}},
    "mem_usage": {"total_vram": {"value": 294896, "unit": "MB"}, "used_vram": {"value": 172032, "unit": "MB"},
                  "free_vram": {"value": 122864, "unit": "MB"}},
}]
_AMD_SMI_STRINGS = {"gpu_data": [{
    "gpu": 3, "usage": {"gfx_activity": "12 %"}, "power": {"socket_power": "250 W"},
    "clock": {"gfx_0": {"clk": "1400 MHz"}}, "temperature": {"edge": "41 C", "hotspot": "N/A"},
    "mem_usage": {"total_vram": "294896 MB", "used_vram": "1024 MB"}}]}


def test_amd_smi_parser_layouts():
    a = nt.parse_amd_smi_metric(json.dumps(_AMD_SMI_DICT_VALUES))[0]
    assert a["busy_percent"] == 93 and a["power_w"] == 987 and a["sclk_mhz"] == 2085
    assert a["vram_total"] == 294896 << 20 and a["vram_used"] == 172032 << 20
    assert a["temp_c"] == {"edge": 50, "hotspot": 72, "mem": 60}
    b = nt.parse_amd_smi_metric(json.dumps(_AMD_SMI_STRINGS))[0]
    assert b["index"] == 3 and b["busy_percent"] == 12 and b["power_w"] == 250 and b["sclk_mhz"] == 1400
    assert b["vram_used"] == 1 << 30 and b["temp_c"] == {"edge": 41}


@pytest.mark.skipif(not os.path.exists(os.path.join(FIX, "amd_smi_metric_mi355x.json")),
                    reason="no captured amd-smi output")
def test_amd_smi_parser_real_mi355x_capture():
    """Output captured from `amd-smi metric --json` on an MI355X box (scripts/capture_telemetry.sh)."""
    with open(os.path.join(FIX, "amd_smi_metric_mi355x.json")) as f:
        g = nt.parse_amd_smi_metric(f.read())
    assert g, "no GPU records parsed"
    r = g[0]
    assert r["vram_total"] and r["vram_total"] > 250 * (1 << 30)  # 288 GB of HBM3E
    assert r["vram_used"] is not None and 0 <= r["vram_used"] <= r["vram_total"]
    assert r["power_w"] is None or 0 < r["power_w"] < 2000


def test_prometheus_lines_reference_names():
    node = {"cpu_percent": 12.5, "cpu_count": 8, "mem_total": 100, "mem_used": 40, "mem_available": 60,
            "shm_used": 1, "disk_total": 10, "disk_used": 4}
    gpus = nt.parse_amd_smi_metric(json.dumps(_AMD_SMI_DICT_VALUES))
    text = "\n".join(nt.prometheus_lines(node, gpus, ip="10.0.0.1", session="s1"))
    assert 'ray_node_cpu_utilization{ip="10.0.0.1",SessionName="s1"} 12.5' in text
    assert 'ray_node_gram_used{ip="10.0.0.1",SessionName="s1",GpuIndex="0",GpuDeviceName="AMD Instinct GPU"} ' \
           f'{172032 << 20}' in text
    assert "ray_node_gpus_utilization{" in text and "ray_node_gpu_power_watts{" in text
    assert 'sensor="hotspot"' in text
    assert "# TYPE ray_node_gram_available gauge" in text


def test_head_metrics_endpoint_has_node_and_gpu_store_gauges(shutdown_only):
    import ray_community_amd as ray

    info = ray.init(num_cpus=2, include_dashboard=True)
    url = (info.get("dashboard_url") if isinstance(info, dict) else getattr(info, "dashboard_url", None))
    assert url
    if not url.startswith("http"):
        url = "http://" + url
    text = urllib.request.urlopen(url + "/metrics", timeout=10).read().decode()
    assert "ray_node_mem_total{" in text and "ray_node_cpu_count{" in text
    assert "rca_gpu_object_store_budget_bytes" in text and "rca_gpu_object_store_spills_total" in text


@pytest.mark.gpu
def test_hbm_gauge_tracks_allocation_gpu(shutdown_only):
    """On the MI355X: ray_node_gram_used (sysfs / amd-smi) rises by an 8 GiB allocation."""
    import re
    import time

    import torch

    import ray_community_amd as ray

    info = ray.init(num_cpus=2, num_gpus=1, include_dashboard=True)
    url = info.get("dashboard_url") if isinstance(info, dict) else getattr(info, "dashboard_url", None)
    url = url if url.startswith("http") else "http://" + url

    def used():
        # node telemetry covers every GPU of the node (sysfs / amd-smi see all of them, the
        # process only its own): {GpuIndex: bytes}
        text = urllib.request.urlopen(url + "/metrics", timeout=10).read().decode()
        vals = {m.group(1): float(m.group(2)) for m in
                re.finditer(r'^ray_node_gram_used\{[^}]*GpuIndex="(\d+)"[^}]*\} (\S+)$', text, re.M)}
        assert vals, "no HBM gauge in /metrics: " + text[:500]
        return vals

    torch.cuda.init()
    torch.cuda.synchronize()
    t0 = time.time()
    while True:  # the first GPU read (visible-GPU resolution through amd-smi) runs in the background
        try:
            before = used()
            break
        except AssertionError:
            if time.time() - t0 > 30:
                raise
            time.sleep(1.0)
    assert len(before) == torch.cuda.device_count(), before  # only this process's GPUs
    x = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    deadline = time.time() + 15
    grew = 0.0
    while time.time() < deadline:
        time.sleep(1.0)
        after = used()
        grew = max(after[k] - before.get(k, after[k]) for k in after)
        if grew >= 7.5 * (1 << 30):
            break
    del x
    assert grew >= 7.5 * (1 << 30), (before, after)


def test_visible_gpu_filter_by_asic_serial(tmp_path):
    """sysfs lists every GPU of the host; only the ones amd-smi reports visible are exported,
    matched by ASIC serial (sysfs unique_id)."""
    for i, uid in enumerate(["aaaa000000000001", "bbbb000000000002", "cccc000000000003"]):
        d = tmp_path / f"card{i * 8}" / "device"
        _w(str(d / "mem_info_vram_total"), str(288 << 30))
        _w(str(d / "mem_info_vram_used"), str((i + 1) << 30))
        _w(str(d / "unique_id"), uid)
    static = {"gpu_data": [{"gpu": 0, "asic": {"asic_serial": "0xCCCC000000000003"}}]}
    serials = nt.parse_amd_smi_serials(static)
    assert serials == ["cccc000000000003"]
    orig = nt._SYSFS_ROOT
    try:
        nt.read_gpus_sysfs.__defaults__ = (str(tmp_path),)
        g = nt.read_gpus(allow_amd_smi=False, serials=serials)
    finally:
        nt.read_gpus_sysfs.__defaults__ = (orig,)
    assert len(g) == 1 and g[0]["index"] == 0 and g[0]["vram_used"] == 3 << 30
    with open(os.path.join(FIX, "amd_smi_static_mi355x.json")) as f:
        assert len(nt.parse_amd_smi_serials(f.read())[0]) == 16  # real capture: 64-bit serial
