"""CPU-side checks of the C-ABI library: it loads, exports every symbol the
header declares, and its layout constants agree with the Python packing."""
import os
import re

import numpy as np

from conftest import REPO


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "nerf_pl_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:NR_EXPORT\s+)?(?:int|int64_t|const char\s*\*)\s+(nr_\w+)\s*\(",
                                 txt, re.M)))


def test_library_exports_header_symbols():
    from nerf_pl_amd import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if getattr(L, s, None) is None]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_layout_constants_match_packing():
    from nerf_pl_amd import ops, packing
    fo, ftot = packing.layer_offsets(packing.FWD_LAYERS)
    bo, btot = packing.layer_offsets(packing.BWD_LAYERS)
    assert ops.layout_query(0) == ftot + packing.HEAD_SIZE == ops.FWD_PACKED
    assert ops.layout_query(1) == ftot
    assert ops.layout_query(2) == btot == ops.BWD_PACKED
    assert ops.layout_query(3) == ops.SAVE_PER_BLOCK
    assert ops.layout_query(4) == ops.GRAD_PER_BLOCK
    assert ops.layout_query(5) == packing.HEAD_SIZE
    assert ops.layout_query(6) == fo["L5"]
    assert ops.layout_query(7) == fo["dir"]
    assert ops.layout_query(8) == bo["L5T"]


def test_packing_maps_are_permutations():
    """Every weight of every packed matrix appears exactly once (fwd), and the
    transposed maps cover exactly the weights the dgrad chain needs."""
    from nerf_pl_amd import packing
    offs, total = packing.param_offsets()
    assert total == 595844
    fm = packing.build_fwd_map()
    used = fm[fm >= 0]
    assert len(np.unique(used)) == len(used) == total
    bm = packing.build_bwd_map()
    assert (bm >= 0).all() and len(np.unique(bm)) == len(bm)
    # transposed maps: dir cols 0..255, final, L8..L6, L5 cols 63.., L4..L2
    exp = []
    for name, (o, shp) in offs.items():
        if not name.endswith("weight") or name in ("sigma.weight", "rgb.0.weight",
                                                   "xyz_encoding_1.0.weight"):
            continue
        r, c = shp
        cols = np.arange(c)
        if name == "dir_encoding.0.weight":
            cols = np.arange(256)
        if name == "xyz_encoding_5.0.weight":
            cols = np.arange(63, c)
        exp.append((o + np.arange(r)[:, None] * c + cols[None, :]).ravel())
    np.testing.assert_array_equal(np.sort(bm), np.sort(np.concatenate(exp)))


def test_pe_pairing_covers_embedding_channels():
    from nerf_pl_amd import packing
    for m, ch in ((packing.PE_MAP, 63), (packing.DIR_MAP, 27)):
        f = m[m >= 0]
        assert sorted(f.tolist()) == list(range(ch))
        # both lane halves of a k-step evaluate the same function (x / sin / cos)
        kind = lambda c: 0 if c < 3 else (1 if (c - 3) % 6 < 3 else 2)  # noqa: E731
        for g in range(m.shape[0]):
            a, b = m[g]
            if a >= 0 and b >= 0:
                assert kind(a) == kind(b)


def test_split_operand_maps_cover_every_weight_once():
    """bf16x6 (3 pieces), f16x3 (2 pieces) and bf16 (1 piece) packed maps: every weight of the
    forward appears once per piece; the transposed maps cover the weights the
    dgrad chain needs, once per piece; sizes match the kernels' buffers."""
    from nerf_pl_amd import packing
    fwd_w = packing.build_fwd_map()
    fwd_w = np.sort(fwd_w[fwd_w >= 0])
    fwd_w = fwd_w[~np.isin(fwd_w, packing.build_fwd3_map(2)[1])]   # head entries
    bwd_w = np.sort(packing.build_bwd_map())
    for np_, fbytes, bbytes in ((3, 3575840, 3342336), (2, 2388000, 2228224),
                                (1, 1200160, 1114112)):
        m, hm = packing.build_fwd3_map(np_)
        assert m.size * 2 + packing.HEAD_BYTES == packing.fwd3_offsets(np_)[1] == fbytes
        used = m[m >= 0]
        assert set(np.unique(used & 3)) == set(range(np_))
        for piece in range(np_):
            w = np.sort(used[(used & 3) == piece] >> 2)
            assert len(np.unique(w)) == len(w)
            np.testing.assert_array_equal(w, fwd_w)
        b = packing.build_bwd3_map(np_)
        assert b.size * 2 == packing.bwd3_bytes(np_) == bbytes
        for piece in range(np_):
            np.testing.assert_array_equal(np.sort(b[(b & 3) == piece] >> 2), bwd_w)
