"""Lines-of-code accounting per component and language.

Counterpart of ``cerebro_gpdb/cloc/run_cloc.sh`` + its file lists: counts
code lines (non-blank, non-comment) of this repository grouped by top-level
component directory and language.

    python -m cerebro_ds_kpgi_amd.tools.loc [--root REPO] [--json out]
"""

import argparse
import collections
import json
import os

LANG = {".py": "Python", ".hip": "HIP", ".h": "C/C++ header", ".cpp": "C++", ".sh": "Shell"}
COMMENT = {"Python": "#", "Shell": "#", "HIP": "//", "C++": "//", "C/C++ header": "//"}
SKIP = {".git", "__pycache__", "build", "gpurun_out", "_lib"}


def count_file(path, lang):
    code = 0
    in_block = False
    pref = COMMENT[lang]
    with open(path, errors="replace") as f:
        for line in f:
            s = line.strip()
            if not s:
                continue
            if pref == "//":
                if in_block:
                    if "*/" in s:
                        in_block = False
                    continue
                if s.startswith("/*"):
                    in_block = "*/" not in s
                    continue
            if s.startswith(pref):
                continue
            code += 1
    return code


def count(root):
    out = collections.defaultdict(lambda: collections.defaultdict(int))
    for d, dirs, files in os.walk(root):
        dirs[:] = [x for x in dirs if x not in SKIP]
        rel = os.path.relpath(d, root)
        parts = rel.split(os.sep)
        comp = parts[0] if parts[0] != "." else "(root)"
        if comp == "cerebro_ds_kpgi_amd" and len(parts) > 1:
            comp = "cerebro_ds_kpgi_amd/" + parts[1]
        for fn in files:
            lang = LANG.get(os.path.splitext(fn)[1])
            if lang:
                out[comp][lang] += count_file(os.path.join(d, fn), lang)
    return {k: dict(v) for k, v in sorted(out.items())}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))))
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    res = count(a.root)
    tot = collections.defaultdict(int)
    for comp, langs in res.items():
        print("{:<36} {}".format(comp, ", ".join("{} {}".format(l, n) for l, n in langs.items())))
        for l, n in langs.items():
            tot[l] += n
    print("{:<36} {}".format("TOTAL", ", ".join("{} {}".format(l, n) for l, n in tot.items())))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"components": res, "total": dict(tot)}, f, indent=1)
    return res


if __name__ == "__main__":
    main()
