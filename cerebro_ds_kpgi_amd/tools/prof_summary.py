"""Summarise a rocprofv3 SQLite output (``--kernel-trace --stats``) as markdown.

    python -m cerebro_ds_kpgi_amd.tools.prof_summary gpurun_out/prof4 [--last-steps K] > profiles/x.md

Groups kernels into the framework's op families (conv fwd/dgrad/wgrad, BN,
pooling, optimizer, loss, data, torch glue) and reports time per step.
``--last-steps K`` keeps only the dispatches of the last K training steps
(step boundaries = the fused Adam kernel, one per step), i.e. the
steady-state HIP-graph replays, excluding init, autotuning and warm-up.
"""

import glob
import os
import re
import sqlite3
import sys

FAMILIES = [
    ("conv/linear GEMM (MFMA, NT: fwd)", r"igemm_nt|pipe_nt"),
    ("conv dgrad (MFMA, NN)", r"igemm_nn_dgrad|igemm_nn32|pipe_nn"),
    ("conv/linear wgrad (MFMA, TN; batched)", r"igemm_wgrad|pipe_wg|wgrad_batch"),
    ("weight transpose (dgrad)", r"transpose_w"),
    ("depthwise conv (fwd / dgrad / wgrad)", r"dw_fwd|dw_dgrad|dw_wgrad"),
    ("batchnorm", r"^bn_|bn_partials|bn_apply|bn_finalize"),
    ("pooling", r"maxpool|gavg|avgpool"),
    ("stem repack / fold", r"stem_"),
    ("bias/act", r"bias_act|bias_grad"),
    ("adam (fused, flat arena)", r"adam"),
    ("softmax-CE + metrics", r"softmax_ce"),
    ("batch gather (HBM store)", r"gather_images"),
    ("memset/copy (runtime)", r"__amd_rocclr|fillBuffer|copyBuffer|cer_fill_kernel"),
    ("torch elementwise glue", r"at::native"),
]


def find_db(path):
    if path.endswith(".db"):
        return path
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit("no .db under {}".format(path))
    return dbs[0]


def _rows(con, last_steps):
    """[(name, calls, total_us, avg_us)] aggregated over the chosen window."""
    disp = list(con.execute("select name, start, end from kernels order by start"))
    if last_steps:
        ends = [e for n, _, e in disp if "adam_kernel" in n]
        if len(ends) > last_steps:
            t0 = ends[-last_steps - 1]
            disp = [d for d in disp if d[1] >= t0 and d[2] <= ends[-1]]
    agg = {}
    for name, st, en in disp:
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += (en - st) / 1000.0
    rows = [(n, c, d, d / c) for n, (c, d) in agg.items()]
    return sorted(rows, key=lambda r: -r[2])


def family(name):
    for label, pat in FAMILIES:
        if re.search(pat, name):
            return label
    return "other"


def _families(rows):
    fam = {}
    for name, calls, dur, avg in rows:
        key = family(name)
        f = fam.setdefault(key, [0, 0.0])
        f[0] += calls
        f[1] += dur
    return fam


def family_ms(path, last_steps):
    """{family: ms per step} over the last ``last_steps`` steps."""
    con = sqlite3.connect(find_db(path))
    fam = _families(_rows(con, last_steps))
    return {k: v[1] / 1000.0 / last_steps for k, v in fam.items()}


def summarize(path, steps=None, title=None, last_steps=None, roofline=None):
    con = sqlite3.connect(find_db(path))
    rows = _rows(con, last_steps)
    if last_steps:
        steps = last_steps
    total = sum(r[2] for r in rows)
    fam = _families(rows)
    out = []
    out.append("# {}".format(title or "rocprofv3 kernel summary"))
    out.append("")
    out.append("source: `{}`; {}total GPU kernel time {:.1f} ms{}".format(
        os.path.relpath(find_db(path)),
        "steady state (last {} steps); ".format(last_steps) if last_steps else "",
        total / 1000.0,
        "" if not steps else " over {} steps = {:.2f} ms/step".format(steps, total / 1000.0 / steps)))
    out.append("")
    out.append("| family | calls | time (ms) | share |")
    out.append("|---|---:|---:|---:|")
    for label, (calls, dur) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        out.append("| {} | {} | {:.2f} | {:.1f}% |".format(label, calls, dur / 1000.0,
                                                         100.0 * dur / total))
    out.append("")
    out.append("## top kernels")
    out.append("")
    out.append("| kernel | calls | total (ms) | avg (us) | share |")
    out.append("|---|---:|---:|---:|---:|")
    for name, calls, dur, avg in rows[:30]:
        short = name if len(name) < 90 else name[:87] + "..."
        out.append("| `{}` | {} | {:.2f} | {:.1f} | {:.1f}% |".format(
            short.replace("|", "\\|"), calls, dur / 1000.0, avg, 100.0 * dur / total))
    text = "\n".join(out) + "\n"
    if roofline and steps:
        from .roofline import roofline_md
        arch, configs, batch, dtype = roofline
        text += "\n" + roofline_md({k: v[1] / 1000.0 / steps for k, v in fam.items()},
                                   arch, configs, batch, dtype)
    return text


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--last-steps", type=int, default=None)
    ap.add_argument("--title", default=None)
    ap.add_argument("--roofline", default=None,
                    help="arch,configs,batch,dtype (e.g. resnet50,8,32,fp32): append a roofline")
    a = ap.parse_args()
    rl = None
    if a.roofline:
        arch, c, b, dt = a.roofline.split(",")
        rl = (arch, int(c), int(b), dt)
    sys.stdout.write(summarize(a.path, a.steps, a.title, a.last_steps, rl))
