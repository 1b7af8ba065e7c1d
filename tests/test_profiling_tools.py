"""scripts/critical_path.py on a synthetic rocpd trace: per-stream busy time, main-stream gaps
and the critical-path window (CPU only)."""
import importlib.util
import os
import sqlite3

HERE = os.path.dirname(os.path.abspath(__file__))


def _tool():
    spec = importlib.util.spec_from_file_location("critical_path", os.path.join(HERE, "..", "scripts",
                                                                                "critical_path.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _db(path, rows):
    c = sqlite3.connect(path)
    c.execute("create table rocpd_info_kernel_symbol (id integer primary key, kernel_name text)")
    c.execute("create table rocpd_kernel_dispatch (kernel_id integer, stream_id integer, queue_id integer, "
              "start integer, end integer)")
    names = {}
    for n, *_ in rows:
        if n not in names:
            names[n] = len(names) + 1
            c.execute("insert into rocpd_info_kernel_symbol values (?, ?)", (names[n], n))
    for n, s, a, b in rows:  # times in us -> ns
        c.execute("insert into rocpd_kernel_dispatch values (?, ?, 0, ?, ?)", (names[n], s, a * 1000, b * 1000))
    c.commit()
    c.close()


def test_critical_path_window_gaps_and_side_streams(tmp_path):
    # (us) step = gemm 0-600, gap 600-700 (side norm kernel busy 550-750), attn 700-900, adamw 900-1000
    rows = []
    for k in range(4):
        o = 1000 * k
        rows += [("gemm", 1, o, o + 600), ("norm", 2, o + 550, o + 750), ("attn", 1, o + 700, o + 900),
                 ("adamw_split_seg_kernel", 1, o + 900, o + 1000)]
    p = str(tmp_path / "t.db")
    _db(p, rows)
    cp = _tool()
    text, span_ms = cp.analyse(cp.load(p), steps=3, marker="adamw")
    assert abs(span_ms - 1.0) < 1e-9  # one step = 1000 us
    lines = {ln.split("|")[1].strip(): ln.split("|")[2].strip() for ln in text.splitlines()
             if ln.startswith("| ") and ln.count("|") == 3}
    assert float(lines["main stream busy (union of its kernels)"]) == 0.90
    assert float(lines["main stream gaps"]) == 0.10
    assert float(lines["-- of which another stream was busy"]) == 0.10
    assert float(lines["-- of which the device was idle"]) == 0
    # the side kernel overlapped 50 us of gemm and 50 ns of attn per step
    assert float(lines["side-stream busy overlapping main-stream kernels"]) == 0.10
    assert "`norm`" in text and "Side-stream kernels" in text
