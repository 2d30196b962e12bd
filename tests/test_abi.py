"""CPU checks of the C-ABI boundary: the library loads and exports every
symbol include/oac_amd.h declares; host-side layout logic (no GPU compute)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "oac_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(oac_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from oac_amd import _lib
    L = _lib.lib()
    decl = declared_functions()
    assert decl, "no declarations parsed"
    missing = [f for f in decl if not hasattr(L, f)]
    assert not missing, missing
    # and the ctypes binding covers exactly the declared surface
    assert sorted(_lib.EXPORTED) == decl


def test_abi_version_and_error_channel():
    from oac_amd import _lib
    L = _lib.lib()
    assert L.oac_abi_version() == 3
    cfg = _lib.SacConfig()
    cfg.kind = 7
    lay = _lib.SacLayout()
    assert L.oac_sac_query_layout(ctypes.byref(cfg), ctypes.byref(lay)) != 0
    assert b"kind" in L.oac_last_error()


@pytest.mark.parametrize("dims", [(376, 17, 256), (111, 8, 256), (1, 1, 256), (11, 3, 32)])
def test_param_layout_matches_reference_parameter_counts(dims):
    """Arena layout covers exactly the reference's parameter counts
    (Humanoid policy 171,042, each critic 166,913)."""
    from oac_amd import _lib, row_layout
    Do, Da, H = dims
    cfg = _lib.SacConfig()
    cfg.kind, cfg.obs_dim, cfg.act_dim, cfg.hidden, cfg.q_out, cfg.batch = 0, Do, Da, H, 1, 256
    for k, v in row_layout(Do, Da).items():
        setattr(cfg, k, v)
    cfg.gemm_cfg = -1
    cfg.world_size = 1
    lay = _lib.SacLayout()
    assert _lib.lib().oac_sac_query_layout(ctypes.byref(cfg), ctypes.byref(lay)) == 0
    n_pol = H * Do + H + H * H + H + 2 * (Da * H + Da)
    n_q = H * (Do + Da) + H + H * H + H + H + 1
    assert lay.pol_size >= n_pol and lay.pol_size - n_pol < 4 * 6
    assert lay.q_size >= n_q and lay.q_size - n_q < 4 * 6
    if dims == (376, 17, 256):
        assert n_pol == 171042 and n_q == 166913
    for f in ("pol_fc0_w", "pol_fc0_b", "pol_fc1_w", "pol_fc1_b", "pol_head_w", "pol_head_b",
              "q_fc0_w", "q_fc0_b", "q_fc1_w", "q_fc1_b", "q_last_w", "q_last_b", "q1_base",
              "q2_base"):
        assert getattr(lay, f) % 4 == 0, f
    assert lay.workspace_floats > 0


def test_row_layout_keeps_critic_input_contiguous():
    from oac_amd import row_layout
    r = row_layout(376, 17)
    assert r["off_act"] == r["off_obs"] + 376
    assert r["row_stride"] % 4 == 0 and r["row_stride"] >= 2 * 376 + 17 + 2


def test_product_path_has_no_fallback(monkeypatch, tmp_path):
    """Without the HIP library every entry point raises (no CPU fallback), and
    the product package never imports the oracle (test infrastructure)."""
    from oac_amd import _lib
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "liboac_amd.so"))
    with pytest.raises(RuntimeError):
        _lib.lib()
    pkg = os.path.join(ROOT, "oac-explore_amd", "oac_amd")
    for f in sorted(os.listdir(pkg)):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert not re.search(r"^\s*(from|import)\s+oracle\b", src, flags=re.M), f
            assert "sac_oracle" not in src, f


def _header_enum(prefix, end):
    """The members of a C enum in include/oac_amd.h, in order (prefix-named)."""
    src = open(os.path.join(ROOT, "include", "oac_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(" + prefix + r"[A-Z0-9_]+)\b\s*(?:=\s*\d+)?\s*,", src)
    return [n for n in dict.fromkeys(names) if n != end]


def test_tuning_keys_match_the_header_and_reject_unknown():
    """oac_amd._lib.TUNE names every oac_tuning_key in the header's order;
    oac_tuning_set takes each key (0 = the default) and rejects one past the
    end with a message (host-only: no GPU call)."""
    from oac_amd import _lib
    keys = _header_enum("OAC_TUNE_", "OAC_TUNE_COUNT")
    assert keys and len(keys) == len(_lib.TUNE)
    py = sorted(_lib.TUNE, key=_lib.TUNE.get)
    assert [k.lower() for k in (n[len("OAC_TUNE_"):] for n in keys)] == py
    L = _lib.lib()
    for name in py:
        _lib.set_tuning(**{name: 0})
    assert L.oac_tuning_set(len(py), 1) != 0
    assert b"tuning key" in L.oac_last_error()


def test_trace_bits_match_the_header():
    """oac_amd._lib.TRACE carries every OAC_TRACE_* bit the header defines."""
    from oac_amd import _lib
    src = open(os.path.join(ROOT, "include", "oac_amd.h")).read()
    bits = {n[len("OAC_TRACE_"):].lower(): int(v)
            for n, v in re.findall(r"#define\s+(OAC_TRACE_[A-Z0-9_]+)\s+(\d+)", src)}
    assert bits == _lib.TRACE
