"""One-screen summary of a bench.py JSON line: per leg value, step time and the edge
kernels' HIP-event times (A/B runs)."""
import json
import sys


def leg(tag, x):
    r = x["roofline"]
    print(f"{tag:11s} {x['value'] / 1e9:7.3f} G/s  {x['ms_per_step']:8.3f} ms  fwd {r['avg_launch_us']:8.1f} us"
          f"  frac {r['frac']:.3f}  {r['kernel']}")
    for k in x.get("edge_kernels", []):
        print(f"             {k['kernel']:34s} {k['avg_us']:8.1f} us  frac {k['frac']:.3f}"
              f"  traffic {k.get('traffic')}")


def main(*paths):
    for path in paths:
        brief(path)


def brief(path):
    text = open(path).read()
    try:  # bench.py --detail file (indented JSON) or a log whose last '{' line is the line
        d = json.loads(text)
    except ValueError:
        d = json.loads([ln for ln in text.splitlines() if ln.startswith("{")][-1])
    leg("head", d)
    for key in ("dropout_p05", "bf16"):
        if key in d:
            leg(key, d[key])
    for key in ("syn2m", "bip1m"):
        for dt, x in d.get(key, {}).items():
            leg(f"{key}_{dt}", x)
    ls = d.get("link_score")
    if ls:
        for pre, x in (("f32", ls), ("bf16", ls.get("bf16"))):
            if not x:
                continue
            print(pre, {k[len("pairs_per_sec_"):]: round(v / 1e9, 3) for k, v in x.items()
                        if k.startswith("pairs_per_sec")}, "allgather_ms", round(x["allgather_ms"], 4))
            for m in ("mlp", "inner"):
                r = x[f"roofline_{m}"]
                mem = r.get("memory", {})
                print(f"   {m:6s} {r['bound']} {r['achieved']:9.1f} {r['unit']} frac {r['frac']:.3f}"
                      f"  {r['avg_launch_us']:8.1f} us  compulsory-HBM frac "
                      f"{mem.get('frac_compulsory_hbm', float('nan')):.3f}  IC frac "
                      f"{mem.get('frac_traffic_ic', float('nan')):.3f}  traffic "
                      f"{mem.get('traffic', r.get('traffic'))}")
    for key in ("train_step_configs1", "train_step_configs2", "train_py_literal"):
        for r in d.get(key, {}).get("runs", []):
            print(f"{key} {r['model']} {r['year']} {r['dtype']}: {r['ms_per_step']:.3f} ms")
    for k, v in d.get("cpu_baseline", {}).items():
        if isinstance(v, dict) and "value" in v:
            print(f"cpu_baseline {k}: {v['value']:.4g} {v['unit']} ({v.get('cores')} cores)")


if __name__ == "__main__":
    main(*sys.argv[1:])
