#!/usr/bin/env python3
"""Per-kernel summary of the SQ PMC passes written by tools/pmc_sq.sh."""
import csv
import sys
from collections import defaultdict


def load(path):
    d = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bd::", "")[:34]
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return d


def main():
    a = load(sys.argv[1])
    b = load(sys.argv[2]) if len(sys.argv) > 2 else {}
    for k, v in a.items():
        wc = v["SQ_WAVE_CYCLES"]
        if wc < 1e6:
            continue
        w = v["SQ_WAVES"]
        line = (f"{k:34s} wait={v['SQ_WAIT_ANY'] / wc:.2f} stall={v['SQ_WAIT_INST_ANY'] / wc:.2f} "
                f"active={v['SQ_ACTIVE_INST_ANY'] / wc:.2f} valu/wave={v['SQ_INSTS_VALU'] / w:.0f} "
                f"lds/wave={v['SQ_INSTS_LDS'] / w:.0f} salu/wave={v['SQ_INSTS_SALU'] / w:.0f}")
        if k in b:
            bv = b[k]
            # SQ_THREAD_CYCLES_VALU: lane-cycles of VALU work; / (64 x ACTIVE_INST_VALU) = lane utilisation
            if bv.get("SQ_ACTIVE_INST_VALU", 0) > 0:
                line += f" lane_util={bv['SQ_THREAD_CYCLES_VALU'] / (64.0 * bv['SQ_ACTIVE_INST_VALU']):.2f}"
        print(line)


if __name__ == "__main__":
    main()
