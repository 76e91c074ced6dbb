"""Error behaviour of the C ABI, checked without a GPU: every compute entry
point validates its sizes and pointers before it touches the device, returns
NR_EINVAL (10001) with a thread-local message naming itself, and treats an
empty problem as a no-op (0, nothing launched).  This mirrors the
reference's only native boundary, torchsearchsorted, which raises on bad
shapes instead of computing (rendering.py:37); the Python wrapper
(_lib.call) turns the code into a RuntimeError carrying the message."""
import pytest

NR_EINVAL = 10001
N = None          # null device pointer
P = 0x10000       # a non-null (never dereferenced) device address


def _cases():
    # (entry, args with a bad size or a null pointer, expected rc)
    c = []
    for sfx in ("", "_x3", "_h3", "_b1"):
        c += [
            (f"nr_mlp_fwd{sfx}", [N, N, N, -1, 8, N, 0, 0, N, N, N], NR_EINVAL),
            (f"nr_mlp_fwd{sfx}", [N, N, N, 0, 8, N, 0, 0, N, N, N], 0),
            (f"nr_mlp_fwd{sfx}", [N, N, N, 5, 8, N, 0, 0, N, N, N], NR_EINVAL),
            (f"nr_mlp_sigma_points{sfx}", [N, N, -1, N, N], NR_EINVAL),
            (f"nr_mlp_sigma_points{sfx}", [N, N, 0, N, N], 0),
            (f"nr_mlp_sigma_points{sfx}", [N, N, 5, N, N], NR_EINVAL),
            (f"nr_mlp_bwd{sfx}", [N, N, N, N, N, -1, N, N], NR_EINVAL),
            (f"nr_mlp_bwd{sfx}", [N, N, N, N, N, 5, N, N], NR_EINVAL),
            (f"nr_wgrad{sfx}", [N, N, -1, N, N, N], NR_EINVAL),
            (f"nr_wgrad{sfx}", [N, N, 5, N, N, N], NR_EINVAL),
        ]
        if True:       # every arithmetic has the sigma-only kernels (fp32 from round 4)
            c += [(f"nr_mlp_bwd_sigma{sfx}", [N, N, N, N, N, -1, N, N], NR_EINVAL),
                  (f"nr_mlp_bwd_sigma{sfx}", [N, N, N, N, N, 0, N, N], 0),
                  (f"nr_mlp_bwd_sigma{sfx}", [N, N, N, N, N, 5, N, N], NR_EINVAL),
                  (f"nr_wgrad_sigma{sfx}", [N, N, -1, N, N, N], NR_EINVAL),
                  (f"nr_wgrad_sigma{sfx}", [N, N, 5, N, N, N], NR_EINVAL)]
        if sfx in ("", "_x3", "_h3"):     # deferred save (not the bf16 variant)
            c += [(f"nr_mlp_fwd_listed{sfx}", [N, N, N, -1, 64, 1, N, N, N, N], NR_EINVAL),
                  (f"nr_mlp_fwd_listed{sfx}", [N, N, N, 0, 64, 1, N, N, N, N], 0),
                  (f"nr_mlp_fwd_listed{sfx}", [N, N, N, 5, 64, 1, N, N, N, N], NR_EINVAL)]
            for so in ("", "_sigma"):
                c += [(f"nr_mlp_bwd{so}_listed{sfx}", [N, N, N, N, N, -1, N, N, N, N], NR_EINVAL),
                      (f"nr_mlp_bwd{so}_listed{sfx}", [N, N, N, N, N, 5, N, N, N, N], NR_EINVAL),
                      (f"nr_wgrad{so}_listed{sfx}", [N, N, -1, N, N, N, N, N], NR_EINVAL),
                      (f"nr_wgrad{so}_listed{sfx}", [N, N, 5, N, N, N, N, N], NR_EINVAL)]
        if sfx in ("", "_x3", "_h3"):     # zero-gradient sample lists (not the bf16 variant)
            for so in ("", "_sigma"):
                c += [(f"nr_mlp_bwd{so}_active{sfx}", [N, N, N, N, N, -1, N, N, N, N], NR_EINVAL),
                      (f"nr_mlp_bwd{so}_active{sfx}", [N, N, N, N, N, 5, N, N, N, N], NR_EINVAL),
                      (f"nr_wgrad{so}_active{sfx}", [N, N, -1, N, N, N, N, N], NR_EINVAL),
                      (f"nr_wgrad{so}_active{sfx}", [N, N, 5, N, N, N, N, N], NR_EINVAL)]
        if sfx:
            c += [(f"nr_pack{sfx}", [N, N, -1, N, N, N], NR_EINVAL),
                  (f"nr_pack_bwd{sfx}", [N, N, -1, N, N], NR_EINVAL)]
    c += [
        ("nr_wgrad_dir_feat", [N, N, N], NR_EINVAL),
        ("nr_active_samples", [N, -1, N, N, N, N], NR_EINVAL),
        ("nr_active_samples", [N, 5, N, N, N, N], NR_EINVAL),
        ("nr_pack", [N, N, -1, N, N], NR_EINVAL),
        ("nr_pack", [N, N, 0, N, N], 0),
        ("nr_pack", [N, N, 7, N, N], NR_EINVAL),
        ("nr_embed", [N, -1, 10, N, N], NR_EINVAL),
        ("nr_embed", [N, 4, 40, N, N], NR_EINVAL),
        ("nr_embed", [N, 0, 10, N, N], 0),
        ("nr_embed", [N, 4, 10, N, N], NR_EINVAL),
        ("nr_coarse_z", [N, N, -1, 64, 0, 1.0, N, 0, N, N], NR_EINVAL),
        ("nr_coarse_z", [N, N, 4, 0, 0, 1.0, N, 0, N, N], NR_EINVAL),
        ("nr_coarse_z", [N, N, 0, 64, 0, 1.0, N, 0, N, N], 0),
        ("nr_coarse_z", [N, N, 4, 64, 0, 1.0, N, 0, N, N], NR_EINVAL),
        ("nr_composite_fwd", [N, 4, 3, N, N, N, 1.0, 0, 1, -1, 64, 0, 0, N, N, N, N, N], NR_EINVAL),
        ("nr_composite_fwd", [N, 4, 3, N, N, N, 1.0, 0, 1, 0, 64, 0, 0, N, N, N, N, N], 0),
        ("nr_composite_fwd", [N, 4, 3, N, N, N, 1.0, 0, 1, 4, 64, 0, 0, N, N, N, N, N], NR_EINVAL),
        ("nr_composite_fwd", [N, 4, 3, N, N, N, 1.0, 0, 1, 4, 0, 0, 0, N, N, N, N, N], NR_EINVAL),
        ("nr_composite_bwd", [N, 4, 3, N, N, N, 1.0, 0, 1, -1, 64, 0, N, N, N, N, N], NR_EINVAL),
        ("nr_composite_bwd", [N, 4, 3, N, N, N, 1.0, 0, 1, 0, 64, 0, N, N, N, N, N], 0),
        ("nr_composite_bwd", [N, 4, 3, N, N, N, 1.0, 0, 1, 4, 64, 0, N, N, N, N, N], NR_EINVAL),
        ("nr_sample_pdf", [N, 2, N, N, N, N, 0, 4, 8, N, N, N], NR_EINVAL),     # < 3 samples
        ("nr_sample_pdf", [N, 64, N, N, N, N, 0, -1, 8, N, N, N], NR_EINVAL),
        ("nr_sample_pdf", [N, 64, N, N, N, N, 0, 0, 8, N, N, N], 0),
        ("nr_sample_pdf", [N, 64, N, N, N, N, 0, 4, 8, N, N, N], NR_EINVAL),
        ("nr_gen_rays", [N, 0, 4, 4, 2.0, 2.0, 1.0, 1.0, 2.0, 0, 1.0, 1.0, 1.0, 2.0, N, 4, N, N,
                         N, N], NR_EINVAL),
        ("nr_gen_rays", [N, 1, 4, 4, 2.0, 2.0, 1.0, 1.0, 2.0, 0, 1.0, 1.0, 1.0, 2.0, N, -1, N, N,
                         N, N], NR_EINVAL),
        ("nr_adam_step", [N, N, N, N, N, -1, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, N], NR_EINVAL),
        ("nr_adam_step", [N, N, N, N, N, 100000, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, N], NR_EINVAL),
        ("nr_mse_loss", [N, N, N, 0, N, N, N], NR_EINVAL),      # the mean of nothing (torch: nan)
        ("nr_mse_loss", [N, N, N, 5, N, N, N], NR_EINVAL),
        ("nr_mse_loss_bwd", [N, N, N, -1, N, N, N, N], NR_EINVAL),
        ("nr_mse_loss_bwd", [N, N, N, 5, N, N, N, N], NR_EINVAL),
        ("nr_opacity_loss", [N, N, N, 9, 8, 0.4, 2000.0, N, N, N], NR_EINVAL),   # n_t > n_o
        ("nr_opacity_loss", [N, N, N, 4, 8, 0.4, 2000.0, N, N, N], NR_EINVAL),
        ("nr_opacity_loss_bwd", [N, 4, 8, 0.4, N, N, N, N, N], NR_EINVAL),
        ("nr_searchsorted", [N, N, 3, 4, 2, 5, 0, N, N], NR_EINVAL),     # 3 vs 2 rows
        ("nr_searchsorted", [N, N, -1, 4, 2, 5, 0, N, N], NR_EINVAL),
        ("nr_searchsorted", [N, N, 0, 4, 0, 5, 0, N, N], 0),
        ("nr_searchsorted", [N, N, 2, 4, 2, 5, 1, N, N], NR_EINVAL),     # null pointers
        ("nr_searchsorted_f64", [N, N, 2, 4, 2, 5, 1, N, N], NR_EINVAL),
        ("nr_sm_normed_depth", [N, N, N, -1, N, N], NR_EINVAL),
        ("nr_sm_normed_depth", [N, N, N, 5, N, N], NR_EINVAL),
        ("nr_sm_normed_depth_bwd", [N, N, N, -1, N, N], NR_EINVAL),
        ("nr_sm_normed_depth_bwd", [N, N, N, 0, N, N], 0),
        ("nr_sm_normed_depth_bwd", [N, N, N, 5, N, N], NR_EINVAL),
        ("nr_sm_backward", [N, N, 1, 1e-3, 1e-3, 0, -1, 16, N, N, N], NR_EINVAL),
        ("nr_sm_backward", [N, N, 1, 1e-3, 1e-3, 0, 4, 0, N, N, N], NR_EINVAL),   # no light map
        ("nr_sm_backward", [N, N, 3, 1e-3, 1e-3, 0, 4, 16, N, N, N], NR_EINVAL),  # bad method
        ("nr_sm_backward", [N, N, 1, 1e-3, 1e-3, 0, 0, 16, N, N, N], 0),
        ("nr_sm_backward", [N, N, 1, 1e-3, 1e-3, 0, 4, 16, N, N, N], NR_EINVAL),  # no output
        ("nr_sm_forward", [N, N, N, N, 0, N, N, N, 128, 128, 2, 1e-3, 1e-3, 0, 1e-5, -1, N, N, N],
         NR_EINVAL),
        # the workspace's 64-bit fixed-point accumulators need an 8-byte aligned base
        ("nr_sm_forward", [P, P, P, P, 0, P, P, P, 8, 8, 2, 1e-3, 1e-3, 0, 1e-5, 4, P + 4, P, N],
         NR_EINVAL),
        ("nr_sm_backward", [P, P + 4, 2, 1e-3, 1e-3, 0, 4, 16, P, P, N], NR_EINVAL),
        # a workspace nr_sm_forward never laid out (its n_light would be unchecked)
        ("nr_sm_backward", [P, P + 0x1000, 2, 1e-3, 1e-3, 0, 4, 16, P, P, N], NR_EINVAL),
    ]
    return c


@pytest.mark.parametrize("entry,args,rc", _cases(), ids=lambda v: v if isinstance(v, str) else None)
def test_entry_point_validates_before_launch(entry, args, rc):
    from nerf_pl_amd import _lib
    L = _lib.lib()
    got = getattr(L, entry)(*args)
    assert got == rc, f"{entry}{tuple(args)} returned {got}: {_lib.last_error()}"
    if rc == NR_EINVAL:
        msg = _lib.last_error()
        base = entry.rsplit("_", 1)[0] if entry[-3:] in ("_x3", "_h3", "_b1") else entry
        assert base in msg, f"{entry}: message {msg!r} does not name the entry point"


def test_python_wrapper_raises_with_message():
    from nerf_pl_amd import _lib
    with pytest.raises(RuntimeError, match=r"nr_embed failed \(code 10001\): nr_embed: bad sizes"):
        _lib.call("nr_embed", None, -1, 10, None, None)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No fallback: without the built library every entry point raises."""
    from nerf_pl_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libnerf_pl_amd.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError, match="HIP library not built"):
        _lib.call("nr_embed", None, 0, 10, None, None)
