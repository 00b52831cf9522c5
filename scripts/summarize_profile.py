"""Condense a scripts/profile.sh output dir into profiles/<tag>/ (committed evidence).

    python scripts/summarize_profile.py gpurun_out/prof_r1 profiles/round1_syn100k [--rev REV]
Writes kernel_stats.csv (rocprofv3 --stats), pmc_summary.json (per-kernel mean of
each counter, with the gfx950 FETCH_SIZE x2 correction applied in a separate field).
"""
import csv
import hashlib
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def files_at_rev(rev, sid):
    """Per-file ids (bench.kernel_source_files) of the sources at git ``rev``, checked
    against the profile's recorded whole-tree id ``sid`` (for profiles whose run recorded
    only the latter)."""
    names = subprocess.run(["git", "ls-tree", "--name-only", "-r", rev, "msha--gnn_amd/csrc",
                            "include"], cwd=ROOT, capture_output=True, text=True,
                           check=True).stdout.split()
    names = sorted(n for n in names if n.endswith((".hip", ".h")) and
                   (n.startswith("include/") or n.count("/") == 2))
    blobs = {n: subprocess.run(["git", "show", f"{rev}:{n}"], cwd=ROOT, capture_output=True,
                               check=True).stdout for n in names}
    h = hashlib.sha256()
    for n in names:  # bench.kernel_source_id's order (sorted paths)
        h.update(os.path.basename(n).encode())
        h.update(blobs[n])
    if h.hexdigest()[:16] != sid:
        raise SystemExit(f"sources at {rev} hash to {h.hexdigest()[:16]}, profile has {sid}")
    return {os.path.basename(n): hashlib.sha256(b).hexdigest()[:16] for n, b in blobs.items()}


def main(src, dst, rev=None):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, "kernel_stats.csv"))
    out = {}
    for d in sorted(os.listdir(src)):
        if not d.startswith("pmc_"):
            continue
        path = os.path.join(src, d, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0]
            e = out.setdefault(k, {})
            c = r["Counter_Name"]
            e.setdefault(c, []).append(float(r["Counter_Value"]))
            e.setdefault("VGPR_Count", r.get("VGPR_Count"))
            e.setdefault("LDS_Block_Size", r.get("LDS_Block_Size"))
    summ = {}
    for k, e in out.items():
        s = {}
        for c, v in e.items():
            if isinstance(v, list):
                s[c] = {"mean": sum(v) / len(v), "n": len(v)}
            else:
                s[c] = v
        if "FETCH_SIZE" in s and "WRITE_SIZE" in s:
            f_kb, w_kb = s["FETCH_SIZE"]["mean"], s["WRITE_SIZE"]["mean"]
            s["hbm_bytes_per_launch_corrected"] = (2 * f_kb + w_kb) * 1024
            s["note"] = ("FETCH_SIZE/WRITE_SIZE in KiB; gfx950 FETCH_SIZE counts half the bytes "
                         "of 16-B/lane streams (MI355X_MICROARCH.md), so fetch is doubled; "
                         "counts L2->fabric traffic incl. Infinity-Cache hits")
        summ[k] = s
    sid = os.path.join(src, "source_id.txt")
    if os.path.exists(sid):  # the sources the profiled library was built from
        summ["_meta"] = {"source_id": open(sid).read().strip()}
        sf = os.path.join(src, "source_files.json")
        if os.path.exists(sf):
            summ["_meta"]["source_files"] = json.load(open(sf))
        elif rev:
            summ["_meta"]["source_files"] = files_at_rev(rev, summ["_meta"]["source_id"])
    json.dump(summ, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    for log in ("bench_trace.log",):
        p = os.path.join(src, log)
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                open(os.path.join(dst, "bench_line.json"), "w").write(lines[-1])
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2],
         sys.argv[sys.argv.index("--rev") + 1] if "--rev" in sys.argv else None)
