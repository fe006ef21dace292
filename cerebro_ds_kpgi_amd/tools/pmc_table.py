"""Per-kernel SQ counter table from rocprofv3 ``--pmc`` CSV runs.

    python -m cerebro_ds_kpgi_amd.tools.pmc_table gpurun_out/pmc_c1/a_X gpurun_out/pmc_c1/b_X

Merges the counter passes of one program (dispatch ids line up because
every pass runs the same launches), keeps our conv kernels, and prints per
kernel: duration, waves, cycles per wave, wait / issue-stall / active
fractions of the wave cycles and instructions per wave.
"""

import collections
import csv
import glob
import os
import sys


def load(dirs):
    per = collections.defaultdict(dict)   # dispatch -> {counter: value, name, dur}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = int(r["Dispatch_Id"])
                    e = per[k]
                    e["name"] = r["Kernel_Name"]
                    e["grid"] = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
                    e["dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
                    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def table(per, pattern="igemm|pipe_|wgrad"):
    import re
    rows = []
    for k, e in sorted(per.items()):
        if not re.search(pattern, e["name"]):
            continue
        w = max(e.get("SQ_WAVES", 1.0), 1.0)
        cyc = e.get("SQ_WAVE_CYCLES", 0.0)
        row = {"kernel": e["name"].split("(")[0][:48], "grid": e["grid"],
               "us": round(e["dur_us"], 1), "waves": int(w),
               "cyc/wave": int(cyc / w) if cyc else None}
        for c, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue-stall"),
                       ("SQ_ACTIVE_INST_ANY", "active")):
            if c in e and cyc:
                row[lab] = round(e[c] / cyc, 2)
        for c, lab in (("SQ_INSTS_MFMA", "mfma/w"), ("SQ_INSTS_VALU", "valu/w"),
                       ("SQ_INSTS_LDS", "lds/w"), ("SQ_INSTS_VMEM_RD", "vmem/w"),
                       ("SQ_INSTS_SALU", "salu/w"), ("SQ_INSTS_SMEM", "smem/w")):
            if c in e:
                row[lab] = round(e[c] / w, 1)
        rows.append(row)
    return rows


def main(argv=None):
    dirs = (argv if argv is not None else sys.argv[1:])
    rows = table(load(dirs))
    if not rows:
        print("no kernels")
        return
    keys = list(rows[0].keys())
    for r in rows:
        for k in r:
            if k not in keys:
                keys.append(k)
    print("| " + " | ".join(keys) + " |")
    print("|" + "---|" * len(keys))
    for r in rows:
        print("| " + " | ".join(str(r.get(k, "")) for k in keys) + " |")


if __name__ == "__main__":
    main()
