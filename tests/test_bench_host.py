"""Host-side pieces of bench.py (no GPU): the C4 graph generator's contract, the
algorithmic byte counts DESIGN.md quotes, and the PMC-traffic lookup of the committed
profiles."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_synth_graph_contract():
    """e unique (row, col) pairs, rows sorted, every row degree >= 1."""
    n, e = 2000, 30000
    rowptr, col = bench.synth_graph(n, e, seed=0)
    assert rowptr[0] == 0 and rowptr[-1] == e and len(col) == e
    deg = np.diff(rowptr)
    assert (deg >= 1).all()
    rows = np.repeat(np.arange(n), deg)
    keys = rows * n + col
    assert (np.diff(keys) > 0).all()  # sorted by (row, col), no duplicates
    assert col.min() >= 0 and col.max() < n
    r2, c2 = bench.synth_graph(n, e, seed=0)
    assert np.array_equal(r2, rowptr) and np.array_equal(c2, col)  # seeded


def test_algorithmic_bytes_match_design():
    """The per-launch byte counts behind the bench's rooflines."""
    n = m = 100_000
    e, H, F = 2_000_000, 8, 16
    assert bench.fwd_bytes(n, m, e, H, F) == 1_154_000_004
    assert bench.fwd_bytes(n, m, e, H, F, s=2) == 616_400_004
    # the fused backward: row stats + column pass + row sum, de in edge order at C4
    nch = m  # one chunk per column at C4
    b = bench.bwd_fused_bytes(n, m, e, H, F, nch)
    assert 1.5e9 < b < 1.7e9
    # de in CSC slot order past 192 MB (edge_attention.hip DE_SLOT_MIN_BYTES) adds the
    # row sum's slot map, 4 B per edge
    def by_hand(E, slot):
        D, s = H * F, 4
        stats = n * (2 * s * D + 8 * H + 12 * H)
        cols = E * (8 + 12 * H + s * D + 4 * H) + m * (2 * s * D + 8 * H) + 12 * nch + 4 * (m + 1)
        return stats + cols + 4 * (n + 1) + E * (4 * H + slot) + n * 4 * H
    assert b == by_hand(e, 0)
    assert bench.bwd_fused_bytes(n, m, 40 * e, H, F, nch) == by_hand(40 * e, 4)
    # with the forward's row terms: no de write, no row sum; the row stats read uc, qc
    # and the row flag and write d_el; the forward writes uc and qc
    D = H * F
    rt = bench.bwd_fused_bytes(n, m, 40 * e, H, F, nch, rowterms=True)
    assert rt == by_hand(40 * e, 4) - 40 * e * 4 * H - (4 * (n + 1) + 40 * e * (4 * H + 4)
                                                        + n * 4 * H) \
        + n * (4 * D + 4 * H + 1 + 4 * H)
    assert bench.fwd_bytes(n, m, e, H, F, 4, True) - bench.fwd_bytes(n, m, e, H, F) == \
        n * (4 * D + 4 * H)


def test_pmc_traffic_only_from_this_build(tmp_path):
    """bench.pmc_lookup attaches PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE per launch) only
    from a profile whose recorded source id is this build's (scripts/profile.sh writes it,
    summarize_profile.py keeps it): the newest such profile wins, a newer profile of
    other sources is skipped and named."""
    import json

    name = "void msha::bip::bip_fwd_kernel<2, 64, float, true, false>"
    pat = r"bip_fwd_kernel<2, 64, float, true, false>"
    entry = {name: {"hbm_bytes_per_launch_corrected": 1.5e9}}
    for tag, sid, val in (("round4_bip1m_v1", bench.kernel_source_id(), 1.5e9),
                          ("round4_bip1m_v2", "0123456789abcdef", 9.9e9)):
        d = tmp_path / tag
        d.mkdir()
        entry[name]["hbm_bytes_per_launch_corrected"] = val
        json.dump(dict(entry, _meta={"source_id": sid}), open(d / "pmc_summary.json", "w"))
    tr, src = bench.pmc_lookup([pat], "*bip1m_v*", profiles_dir=str(tmp_path))
    assert tr == 1.5e9 and src.endswith("round4_bip1m_v1/pmc_summary.json")
    (tmp_path / "round4_bip1m_v1" / "pmc_summary.json").unlink()
    tr, src = bench.pmc_lookup([pat], "*bip1m_v*", profiles_dir=str(tmp_path))
    assert tr is None and "other sources" in src
    assert len(bench.kernel_source_id()) == 16


def test_pmc_traffic_per_file_identity(tmp_path):
    """A profile of another whole-tree id still serves a kernel whose defining file and
    every header are unchanged (_meta.source_files), and no kernel whose file changed."""
    import json

    files = bench.kernel_source_files()
    assert bench._kernel_defs()["bip_fwd_kernel"] == "edge_bip.hip"
    bip = "void msha::bip::bip_fwd_kernel<2, 64, float, true, false>"
    pair = "void msha::sk::pair_x3_kernel<128, 128, 3>"
    d = tmp_path / "round4_link_v1"
    d.mkdir()
    edited = dict(files, **{"edge_bip.hip": "0" * 16})
    json.dump({bip: {"hbm_bytes_per_launch_corrected": 1e9},
               pair: {"hbm_bytes_per_launch_corrected": 2e9},
               "_meta": {"source_id": "0123456789abcdef", "source_files": edited}},
              open(d / "pmc_summary.json", "w"))
    tr, src = bench.pmc_lookup([r"pair_x3_kernel<"], "*link*", profiles_dir=str(tmp_path))
    assert tr == 2e9
    tr, src = bench.pmc_lookup([r"bip_fwd_kernel<"], "*link*", profiles_dir=str(tmp_path))
    assert tr is None and "other sources" in src
    hdr = dict(files, **{"common.h": "0" * 16})  # a header change invalidates every kernel
    json.dump({pair: {"hbm_bytes_per_launch_corrected": 2e9},
               "_meta": {"source_id": "0123456789abcdef", "source_files": hdr}},
              open(d / "pmc_summary.json", "w"))
    tr, _ = bench.pmc_lookup([r"pair_x3_kernel<"], "*link*", profiles_dir=str(tmp_path))
    assert tr is None


def test_gpus_flag_launches_ranks():
    """``bench.py --gpus 2`` without WORLD_SIZE starts two ranks itself (torch.distributed.run
    on 127.0.0.1); --dry-run runs them over gloo on the CPU: both ranks report, the sharded
    table all-gathers exactly and the pair split covers the batch."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_reporting"] == 2 and d["table_ok_ranks"] == 2
    assert d["pairs_covered"] == d["pairs"]


def test_dry_run_world4_records_the_ranks():
    """``--gpus 4 --dry-run`` (gloo, CPU): the line records the process group's world
    size and backend and one census entry per rank (RANK / LOCAL_RANK / device), the
    fields a driver's 8-GPU run uses to prove how many ranks RCCL formed."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["world_size"] == 4 and d["backend"] == "gloo"
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1, 2, 3]
    assert sorted(x["local_rank"] for x in d["ranks"]) == [0, 1, 2, 3]
    assert d["ranks_reporting"] == 4 and d["table_ok_ranks"] == 4
    assert d["pairs_covered"] == d["pairs"] and d["exchange"] == "gloo"


def test_gpus_flag_mismatch_fails():
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0


def _maximal_out():
    """The round-4 builder line (every leg present, 23 KB) widened to 8 ranks with a NaN
    and an infinity planted: the largest dict main() can hand to compact_line."""
    import copy
    import json

    d = json.load(open(os.path.join(ROOT, "profiles", "round4_final", "bench_line.json")))
    d = copy.deepcopy(d)
    r0 = d["ranks"]["ranks"][0]
    d["ranks"] = {"world_size": 8, "backend": "nccl (RCCL)",
                  "ranks": [dict(r0, rank=i, local_rank=i, device=f"cuda:{i}",
                                 pci_bus_id=f"0000:{0x10 + i:02x}:00") for i in range(8)]}
    d["roofline"]["traffic"] = float("nan")
    d["bip1m"]["f32"]["roofline"]["frac"] = float("inf")
    return d


def test_bench_line_is_small_strict_json():
    """the stdout line stays <= 12 KB, is strict JSON (no NaN/Infinity
    tokens) and carries the contract keys, roofline, cpu_baseline and the compact legs."""
    import json

    out = _maximal_out()
    s = bench.dumps_line(bench.compact_line(out, "gpurun_out/bench_detail.json"))
    assert "\n" not in s
    assert len(s.encode()) <= bench.LINE_MAX_BYTES, len(s)
    assert len(s.encode()) <= 8 * 1024  # the driver's stdout tail

    def bad(tok):
        raise ValueError(tok)

    line = json.loads(s, parse_constant=bad)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype",
              "config", "ranks", "roofline", "cpu_baseline", "legs", "higher_is_better",
              "scaling", "vs_baseline", "data"):
        assert k in line, k
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    assert line["roofline"]["traffic"] is None  # the planted NaN
    assert len(line["ranks"]["ranks"]) == 8
    legs = line["legs"]
    for k in ("c4_f32", "c4_bf16", "syn2m_f32", "syn2m_bf16", "bip1m_f32", "bip1m_bf16",
              "link_mlp_f32", "link_inner_bf16_overlapped", "step_Ours_2015_f32",
              "step_ablation3_2015_f32", "step_Ours_2018_bf16", "trainpy_Ours"):
        assert k in legs, k
    assert legs["bip1m_f32"]["frac"] is None  # the planted infinity
    assert {"value", "unit", "cores", "kind", "sample"} <= set(line["cpu_baseline"])


def test_bip_kernel_patterns_match_rocprof_names():
    """The bipartite rooflines' PMC lookup names every kernel family (the MFMA kernels of
    edge_bip3.hip, the mask kernels of edge_bip2.hip and the CSR walk of edge_bip.hip) as
    rocprofv3 reports them: fp32
    demangled, bf16 mangled (DF16b) or demangled with the type as "bool _Accum"."""
    import re

    fwd, bwd = bench.bip_kernel_patterns(2, 64, False, True)
    names_f = ["void msha::bip2::bip2_fwd_kernel<float, true, false>(unsigned int const*)",
               "void msha::bip::bip_fwd_kernel<2, 64, float, true, false, 2>(int const*)",
               "void msha::bip3::bip3_fwd_kernel<float, true, false, false>(unsigned int const*)"]
    names_b = ["void msha::bip2::bip2_bwd_kernel<float, true, false, false>(unsigned int const*)",
               "void msha::bip::bip_bwd_kernel<2, 64, float, true, true, 2>(int const*)",
               "void msha::bip3::bip3_bwd_kernel<float, true, false, false>(unsigned int const*)"]
    assert all(re.search(fwd, n) for n in names_f) and not any(re.search(fwd, n) for n in names_b)
    assert all(re.search(bwd, n) for n in names_b) and not any(re.search(bwd, n) for n in names_f)
    # the v branch (HS) is pinned: a u-only forward is another instantiation
    assert not re.search(fwd, "void msha::bip2::bip2_fwd_kernel<float, false, false>(unsigned")
    fwd16, bwd16 = bench.bip_kernel_patterns(2, 64, True, True)
    assert re.search(fwd16, "_ZN4msha4bip215bip2_fwd_kernelIDF16bLb1ELb0EEEvPKjPKiPKh")
    assert re.search(fwd16, "void msha::bip2::bip2_fwd_kernel<bool _Accum, bool, E, false>")
    assert re.search(bwd16, "_ZN4msha4bip215bip2_bwd_kernelIDF16bLb1ELb0ELb0EEEv")
    # the MFMA kernels (edge_bip3.hip), as rocprofv3 printed them in profiles/round6_bip_sq
    assert re.search(fwd16, "void msha::bip3::bip3_fwd_kernel<bool _Accum, bool, E, false, false>(")
    assert re.search(bwd16, "void msha::bip3::bip3_bwd_kernel<bool _Accum, bool, E, false, false>(")
    assert not re.search(bwd16, "void msha::bip3::bip3_fwd_kernel<bool _Accum, bool, E, false, false>(")
    assert not re.search(fwd16, "void msha::bip2::bip2_fwd_kernel<float, true, false>(")
