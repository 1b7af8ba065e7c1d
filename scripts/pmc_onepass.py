"""One rocprofv3 --pmc pass (8 SQ counters + GRBM_GUI_ACTIVE) summarised per kernel: duration,
MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), the wave-cycle
split wait / issue-stall / active, LDS issue stalls and bank-conflict share.

    python scripts/pmc_onepass.py <rocprofv3 -d dir>
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load, short  # noqa: E402


def main():
    A = load(sys.argv[1])
    print("| kernel | n | avg us | MFMA util | wait | issue stall | of which LDS | active | LDS confl/active |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k in sorted(A, key=lambda k: -A[k]["_t"]):
        a = A[k]
        n = a["_n"]
        wc = a.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        grbm = a.get("GRBM_GUI_ACTIVE", 0.0)
        mfma = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (grbm / 8 * 1024) if grbm else 0.0
        lds = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_LDS_IDX_ACTIVE"] if a.get("SQ_LDS_IDX_ACTIVE") else 0.0
        print(f"| `{short(k, 70)}` | {int(n)} | {a['_t'] / n * 1e6:.1f} | {mfma * 100:.1f}% | "
              f"{a.get('SQ_WAIT_ANY', 0) / wc * 100:.1f}% | {a.get('SQ_WAIT_INST_ANY', 0) / wc * 100:.1f}% | "
              f"{a.get('SQ_WAIT_INST_LDS', 0) / wc * 100:.1f}% | {a.get('SQ_ACTIVE_INST_ANY', 0) / wc * 100:.1f}% | "
              f"{lds * 100:.1f}% |")


if __name__ == "__main__":
    main()
