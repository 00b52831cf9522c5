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


def main(path):
    lines = [ln for ln in open(path) if ln.startswith("{")]
    d = json.loads(lines[-1])
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
                print(f"   {m:6s} {r['bound']} {r['achieved']:9.1f} {r['unit']} frac {r['frac']:.3f}"
                      f"  {r['avg_launch_us']:8.1f} us  traffic {r.get('traffic')}")
    for key in ("train_step_configs1", "train_step_configs2"):
        for r in d.get(key, {}).get("runs", []):
            print(f"{key} {r['model']} {r['year']} {r['dtype']}: {r['ms_per_step']:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
