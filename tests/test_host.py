"""CPU-side checks of the host layer: ABI surface, drop-in constructors, graph plans.

No compute call reaches the GPU here (these run in the CPU-only container)."""
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT, golden


def header_symbols():
    text = open(os.path.join(ROOT, "include", "msha_gnn.h")).read()
    return sorted(set(re.findall(r"MSHA_API\s+[\w\s\*]+?\b(msha_\w+)\s*\(", text)))


def test_header_symbols_bound_by_ctypes(msha):
    from msha_gnn_amd import _lib

    assert header_symbols() == _lib.exported_symbols()


def test_library_exports_every_header_symbol(msha):
    from msha_gnn_amd import _lib

    lib = _lib.load()  # loads without touching the GPU
    assert lib.msha_abi_version() == _lib.ABI_VERSION == 16
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (msha_\w+)", out))
    assert set(header_symbols()) <= exported
    # host-only queries (no kernel launch)
    assert lib.msha_edge_attention_supported(8, 16) == 1
    assert lib.msha_edge_attention_supported(3, 16) == 0
    assert lib.msha_graph_workspace_size(39179, 32) > 0
    # model head: R15's shape (2 heads x 64, 32 recipients) is covered, 9 heads are not
    assert lib.msha_head_supported(32, 2, 64) == 1
    assert lib.msha_head_supported(32, 9, 64) == 0
    assert lib.msha_head_supported(300, 2, 64) == 0


def test_abi_argument_errors_are_reported(msha):
    from msha_gnn_amd import _lib

    with pytest.raises(RuntimeError, match="graph descriptor is NULL"):
        _lib.call("msha_edge_attention_fwd", None, 8, 16, 0, None, None, None, 0.2, 0.0, 0, 0,
                  None, None, None, None, None)
    with pytest.raises(RuntimeError, match="p must be in"):
        _lib.call("msha_dropout_keep_mask", 0, 0, 10, 1.5, 1, None)


def _sd_equal(a, b_npz, prefix):
    for k, v in a.items():
        ref = b_npz[prefix + k]
        assert np.array_equal(v.numpy(), ref), k


def test_ablation3_init_matches_reference_bitwise(msha):
    from msha_gnn_amd import layers

    z = golden("sub512.npz")
    gdp = {i: float(x) for i, x in enumerate(z["gdp"])}
    torch.manual_seed(0)
    m = layers.ablation3(in_features=128, out_features=64, n_classes=32, n_heads=2, dropout=0.0,
                         gdp=gdp, Scount=512, Rcount=32)
    sd = m.state_dict()
    assert list(sd.keys()) == [k[len("init."):] for k in z.files if k.startswith("init.")]
    _sd_equal(sd, z, "init.")


def test_gat_init_matches_reference_bitwise(msha):
    from msha_gnn_amd import layers

    z = golden("gat_sub512.npz")
    s = golden("sub512.npz")
    gdp = {i: float(x) for i, x in enumerate(s["gdp"])}
    torch.manual_seed(1)
    m = layers.GAT(n_features=32, n_classes=32, n_heads=2, dropout=0.0, gdp=gdp, N=512)
    sd = m.state_dict()
    assert list(sd.keys()) == [k[len("init."):] for k in z.files if k.startswith("init.")]
    _sd_equal(sd, z, "init.")


def test_ours_layer3_init_matches_reference(msha):
    from msha_gnn_amd import layers

    e = golden("edge_cases.npz")
    torch.manual_seed(6)
    layer = layers.OursLayer3(16, 8, 0.0)
    _sd_equal(layer.state_dict(), e, "ol3.init.")
    torch.manual_seed(8)
    gal = layers.GraphAttentionLayer(20, 80, 0.0)
    _sd_equal(gal.state_dict(), e, "gal.init.")


def test_csc_chunk_plan(msha):
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(0)
    n, m = 3000, 7
    deg = rng.integers(1, 5, n)
    rowptr = np.concatenate([[0], np.cumsum(deg)])
    col = np.concatenate([np.sort(rng.choice(m, d, replace=False)) for d in deg])
    col[rowptr[:-1]] = 0  # column 0 is long: >= 3000 slots -> several chunks
    col = np.concatenate([np.unique(col[rowptr[i]:rowptr[i + 1]]) for i in range(n)])
    rowptr = np.concatenate([[0], np.cumsum([len(np.unique(col[rowptr[i]:rowptr[i + 1]]))
                                             for i in range(n)])])
    g = Graph.from_csr(rowptr, col, m, device="cpu")
    p = g._plan
    colptr = g.colptr.numpy()
    cc, cs, ce = p["chunk_col"].numpy(), p["chunk_start"].numpy(), p["chunk_end"].numpy()
    # chunks tile every column's CSC range in order, each <= CSC_CHUNK slots
    for j in range(m):
        sel = np.nonzero(cc == j)[0]
        assert cs[sel[0]] == colptr[j] and ce[sel[-1]] == colptr[j + 1]
        assert np.all(cs[sel[1:]] == ce[sel[:-1]]) and np.all(ce[sel] - cs[sel] <= 512)
    mc = p["multi_col"].numpy()
    assert 0 in mc and np.all(p["multi_count"].numpy() > 1)
    # CSC slots: ascending rows within a column, eids map back to the same (row, col)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    cr, ceid = g.csc_row.numpy(), g.csc_eid.numpy()
    assert np.array_equal(rows[ceid], cr)
    for j in range(m):
        seg = cr[colptr[j]:colptr[j + 1]]
        assert np.all(np.diff(seg) > 0) and np.all(col[ceid[colptr[j]:colptr[j + 1]]] == j)


def test_ops_refuse_cpu_tensors(msha):
    from msha_gnn_amd import layers

    torch.manual_seed(0)
    gal = layers.GraphAttentionLayer(4, 3, 0.0)
    with pytest.raises(RuntimeError, match="GPU only"):
        gal(torch.rand(5, 4), torch.ones(5, 3))


def test_gcn_init_bit_identical(msha):
    """layers.GCN (model.py:48-55) after the fixture's seed: same keys, shapes, values
    (scalar biases included)."""
    from conftest import golden
    from msha_gnn_amd import layers

    z = golden("gcn_sub512.npz")
    s = golden("sub512.npz")
    gdp = {i: float(x) for i, x in enumerate(s["gdp"])}
    torch.manual_seed(4)
    model = layers.GCN(nfeat=64, nhid=128, nclass=32, dropout=0.0, gdp=gdp, N=512)
    sd = model.state_dict()
    assert sorted(sd) == sorted(k[len("init."):] for k in z.files if k.startswith("init."))
    for k, v in sd.items():
        assert np.array_equal(v.numpy(), z["init." + k]), k


def test_from_csr_records_what_the_bipartite_kernels_need(msha):
    """Graph.from_csr notes duplicate columns in a row and the largest row degree on the
    host; functional.bip_ok keeps such graphs off the bipartite kernels (rows with
    distinct columns, at most 64 / heads each)."""
    import numpy as np

    from msha_gnn_amd.graph import Graph

    g = Graph.from_csr(np.array([0, 2, 3]), np.array([1, 1, 0]), 4, "cpu")
    assert (g.distinct_cols, g.max_deg) == (False, 2)
    g = Graph.from_csr(np.array([0, 2, 5]), np.array([1, 3, 0, 2, 3]), 4, "cpu")
    assert (g.distinct_cols, g.max_deg) == (True, 3)


def test_segment_records_pack_as_the_struct(msha):
    """_segments' packed records (struct.pack_into) are byte-identical to ctypes
    MshaSegment records built field by field."""
    import ctypes

    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF

    rec = (0x7f0012345600, 0x7f0012349900, 17, 129, 129, 256, None, 0, 0.5, 2**61 + 3,
           torch.bfloat16, torch.float32)
    a, dst, rows, cols, lda, ldd, b, ldb, p, seed, adt, ddt = rec
    ref = _lib.MshaSegment(a, b, dst, rows, cols, lda, ldb, ldd, p, seed, 0, 1, 0)
    buf = bytearray(MF._SEG_FMT.size)
    MF._SEG_FMT.pack_into(buf, 0, a, b or 0, dst, rows, cols, lda, ldb, ldd, p, seed, 0, 1, 0)
    assert bytes(buf) == ctypes.string_at(ctypes.addressof(ref), ctypes.sizeof(ref))


def _bf16(x):
    """Round fp32 -> bf16 (round to nearest even), returned as fp32 (numpy emulation of
    v_cvt_pk_bf16_f32 for finite values)."""
    import numpy as np

    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def test_split_bf16_products_reach_fp32_accuracy():
    """The split-bf16 fp32 GEMM scheme of skinny.hip (pair_x3_kernel, the split proj_kernel):
    x = x_h + x_m + x_l with x_h = bf16(x), x_m = bf16(x - x_h), x_l = bf16(x - x_h - x_m);
    the six products hh, hm, mh, mm, hl, lh summed in fp32 give each product within a few
    fp32 ulps, and a 128-term dot within the fp32 forward-error bound of the exact-fp32
    MFMA (n 2^-24 sum|x w|)."""
    import numpy as np

    rng = np.random.default_rng(0)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-8, 8, 200000))).astype(np.float32)
    w = (rng.standard_normal(200000) * np.exp(rng.uniform(-8, 8, 200000))).astype(np.float32)

    def split(a):
        h = _bf16(a)
        r1 = (a - h).astype(np.float32)  # exact in fp32
        m = _bf16(r1)
        r2 = (r1 - m).astype(np.float32)  # exact in fp32
        return h, m, _bf16(r2)

    xh, xm, xl = split(x)
    wh, wm, wl = split(w)
    # the three terms carry x to 2^-27 of |x| (fp32 has 24 bits)
    assert np.all(np.abs((xh.astype(np.float64) + xm + xl) - x) <= 2.0 ** -26 * np.abs(x))
    # each bf16 x bf16 product is exact in fp32
    for a, b in ((xh, wh), (xm, wl), (xl, wm)):
        assert np.array_equal((a * b).astype(np.float64), a.astype(np.float64) * b)
    # six products (small terms first, as the kernels order them), fp32 accumulation
    terms = (xl * wh, xh * wl, xm * wm, xh * wm, xm * wh, xh * wh)
    acc = np.zeros_like(x)
    for t in terms:
        acc = (acc + t).astype(np.float32)
    exact = x.astype(np.float64) * w.astype(np.float64)
    rel = np.abs(acc - exact) / np.abs(exact)
    assert rel.max() <= 2.0 ** -21, rel.max()  # a few fp32 ulps (the dropped ml, lm, ll)
    # a 128-term dot product accumulated sequentially in fp32 in the kernels' order (per k,
    # the six products small terms first): within the exact-fp32 dot's n u A bound with
    # n = 128 -- the 768 split terms add no more error than the 128 fp32 products would
    X = x[:128 * 1000].reshape(1000, 128)
    Wv = w[:128 * 1000].reshape(1000, 128)
    sX, sW = split(X), split(Wv)
    pairs = ((2, 0), (0, 2), (1, 1), (0, 1), (1, 0), (0, 0))  # lh, hl, mm, hm, mh, hh
    dot = np.zeros(1000, np.float32)
    for k in range(128):
        for i, j in pairs:
            dot = (dot + (sX[i][:, k] * sW[j][:, k]).astype(np.float32)).astype(np.float32)
    ref = (X.astype(np.float64) * Wv.astype(np.float64)).sum(1)
    bound = 128 * 2.0 ** -24 * (np.abs(X.astype(np.float64) * Wv)).sum(1)
    assert np.all(np.abs(dot - ref) <= bound)


def test_adam_rejects_loaded_unsupported_flags(msha):
    """a torch.optim.Adam state_dict saved with amsgrad / maximize must not
    silently run plain Adam after load_state_dict."""
    import pytest
    import torch

    from msha_gnn_amd.optim import Adam

    p = torch.nn.Parameter(torch.zeros(4))
    ref = torch.optim.Adam([torch.nn.Parameter(torch.zeros(4))], amsgrad=True)
    opt = Adam([p])
    with pytest.raises(NotImplementedError, match="amsgrad"):
        opt.load_state_dict(ref.state_dict())
