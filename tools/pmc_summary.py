#!/usr/bin/env python
"""Per-kernel utilisation summary from rocprofv3 --pmc passes (tools/gpu_job.sh pmc_* steps).

    python tools/pmc_summary.py gpurun_out/pmc_attn1 gpurun_out/pmc_attn2 [name-filter]

Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles;
SQ_VALU_MFMA_BUSY_CYCLES = 32 x the 32x32x16 MFMAs; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import collections
import csv
import sys

csv.field_size_limit(1 << 30)


def main():
    dirs = [a for a in sys.argv[1:] if "/" in a]
    filt = [a for a in sys.argv[1:] if "/" not in a]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in dirs:
        for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
            k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if filt and not any(f in k for f in filt):
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        if "GRBM_GUI_ACTIVE" not in v or "SQ_WAVE_CYCLES" not in v:
            continue
        T = v["GRBM_GUI_ACTIVE"] / 8
        wc = v["SQ_WAVE_CYCLES"]
        out = [f"{k[:44]:44s}", f"mfma {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (T * 1024):.3f}",
               f"waves/CU {wc * 4 / T / 256:.2f}", f"wait {v['SQ_WAIT_ANY'] / wc:.2f}",
               f"issue {v['SQ_ACTIVE_INST_ANY'] / wc:.2f}", f"valu-act {v['SQ_ACTIVE_INST_VALU'] / wc:.2f}",
               f"lds-act {v['SQ_ACTIVE_INST_LDS'] / wc:.2f}", f"lds-wait {v['SQ_WAIT_INST_LDS'] / wc:.2f}"]
        if v.get("SQ_INSTS_MFMA"):
            m = v["SQ_INSTS_MFMA"]
            out += [f"valu/mfma {v['SQ_INSTS_VALU'] / m:.1f}", f"lds/mfma {v['SQ_INSTS_LDS'] / m:.2f}",
                    f"salu/mfma {v['SQ_INSTS_SALU'] / m:.2f}", f"bank-confl {v.get('SQ_LDS_BANK_CONFLICT', 0):.3g}"]
        print("  ".join(out))


if __name__ == "__main__":
    main()
