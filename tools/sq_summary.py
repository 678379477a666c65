"""Summarise tools/nn_pmc.sh's rocprofv3 passes (gpurun_out/npmc, k_resnet on
tools/nn_ablation.py's 4096-row launches) into profiles/<tag>_resnet_sq.json:
per-launch counter averages and the derived wave-state / LDS fractions
(SQ_WAVE_CYCLES, SQ_WAIT_* and SQ_ACTIVE_* count quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES cycles; MI355X_MICROARCH.md 'rocprofv3 PMC slots').

Usage: python tools/sq_summary.py <tag> [source note]
"""

import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main(tag: str, source: str) -> None:
    acc = defaultdict(list)
    for f in glob.glob(str(ROOT / "gpurun_out" / "npmc" / "**" / "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_resnet" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())}
    cycles = c["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
    wave = c["SQ_WAVE_CYCLES"]
    d = {
        "cycles_per_launch": round(cycles),
        "mfma_busy_frac": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * cycles), 4),
        "mfma_insts_per_launch": float(c["SQ_INSTS_MFMA"]),
        "wave_parked_frac (SQ_WAIT_ANY: s_waitcnt / s_barrier)": round(c["SQ_WAIT_ANY"] / wave, 4),
        "wave_issue_stalled_frac (SQ_WAIT_INST_ANY: MFMA pipe held by the partner / RAW)":
            round(c["SQ_WAIT_INST_ANY"] / wave, 4),
        "wave_issuing_frac (SQ_ACTIVE_INST_ANY)": round(c["SQ_ACTIVE_INST_ANY"] / wave, 4),
        "lds_issue_stall_frac (SQ_WAIT_INST_LDS)": round(c["SQ_WAIT_INST_LDS"] / wave, 4),
        "lds_array_busy_frac (SQ_LDS_IDX_ACTIVE / (256 CUs x cycles))": round(c["SQ_LDS_IDX_ACTIVE"] / (256 * cycles), 4),
        "lds_bank_conflict_frac_of_lds_cycles": round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4),
        "valu_insts_per_mfma (SQ_INSTS_VALU includes MFMA)": round(c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"], 3),
        "non_mfma_valu_per_mfma": round(c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"] - 1, 3),
        "salu_insts_per_mfma": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_MFMA"], 3),
        "lds_insts_per_mfma": round(c["SQ_INSTS_LDS"] / c["SQ_INSTS_MFMA"], 3),
    }
    out = {"tag": tag, "source": source, "counters_per_launch": c, "derived": d}
    (ROOT / "profiles" / f"{tag}_resnet_sq.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(d))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else
         "tools/nn_pmc.sh over tools/nn_ablation.py (k_resnet_w8, 4096 rows, 128x10b bf16, f32 input path), "
         "4 rocprofv3 --pmc passes, per-launch averages")
