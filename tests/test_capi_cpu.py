"""CPU-side checks of the C-ABI library (no GPU calls): it loads, exports every
symbol include/cvae.h declares, and its host-only planner agrees with the
reference's parameter layout (Training_VAE.py:132-167)."""
import os

import pytest
import torch

from conftest import ROOT
from oracle.cvae_oracle import OracleCVAE


@pytest.fixture(scope="module")
def cl():
    from cvae_amd import _build, _lib
    _build.build()
    return _lib


def test_library_exports_every_header_symbol(cl):
    names = cl.header_symbols(os.path.join(ROOT, "include", "cvae.h"))
    assert len(names) >= 15
    L = cl.lib()
    for n in names:
        assert hasattr(L, n), n
    assert L.cvae_abi_version() == 3
    assert cl.missing_signatures(os.path.join(ROOT, "include", "cvae.h")) == []  # ctypes covers the whole ABI


@pytest.mark.parametrize("S,D,Z,H,dtype", [(10, 3, 8, 128, "fp32"), (100, 6, 8, 128, "bf16"),
                                           (100, 6, 8, 128, "fp32"), (10, 3, 8, 16, "fp32"),
                                           (10, 3, 8, 16, "bf16"), (50, 4, 16, 64, "bf16")])
def test_param_layout_matches_state_dict(cl, S, D, Z, H, dtype):
    from cvae_amd import config_info
    n, nt, lds = config_info(S, D, Z, H, dtype=dtype)
    ref = OracleCVAE(S, D, Z, H)
    assert nt == len(ref.state_dict()) == 24
    assert n == sum(p.numel() for p in ref.parameters())
    assert 0 < lds <= 160 * 1024


def test_known_param_counts(cl):
    from cvae_amd import config_info
    assert config_info(10, 3, 8)[0] == 128942      # SURVEY §2 (measured on the reference)
    assert config_info(100, 6, 8)[0] == 275432


def test_unsupported_config_reports_error(cl):
    from cvae_amd import config_info
    from cvae_amd._lib import CvaeError
    with pytest.raises(CvaeError, match="LDS"):
        config_info(1000, 6, 2048, 128, 8, 8, dtype="bf16")
    with pytest.raises(CvaeError, match="dim"):
        config_info(10, 2, 8)


def test_wide_cfg5_config_plans(cl):
    """BASELINE cfg5's shape (S=200, Z=512, 8+8 layers) plans with a smaller row tile: its tile
    state fits 160 KiB of LDS with 8 rows (bf16) / 4 rows (fp32), not 16."""
    from cvae_amd import config_info
    for dt in ("bf16", "fp32", "fp8"):
        n, nt, lds = config_info(200, 6, 512, 128, 8, 8, dtype=dt)
        assert nt == 2 * (2 + 8 + 2 + 8) and 0 < lds <= 160 * 1024
        H, I, Z = 128, 1200, 512
        want = (2 * H + H) + (H * H + H) + (I * H + H) + 7 * (H * H + H) + 2 * (2 * H * Z + Z) \
            + ((Z + H) * H + H) + 6 * (H * H + H) + (H * I + I)
        assert n == want


def test_engine_refuses_without_gpu(cl):
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cvae_amd import ConditionalTrajectoryVAE, CVAEEngine
    with pytest.raises(RuntimeError, match="HIP device"):
        CVAEEngine(10, 3, 8)
    m = ConditionalTrajectoryVAE(10, 3, 8)
    with pytest.raises(RuntimeError, match="attach"):
        m(torch.zeros(2, 10, 3), torch.zeros(2, 2))


def test_model_init_and_state_dict_match_reference_layout(cl):
    from cvae_amd import ConditionalTrajectoryVAE
    torch.manual_seed(0)
    a = ConditionalTrajectoryVAE(10, 3, 8)
    torch.manual_seed(0)
    b = OracleCVAE(10, 3, 8)
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa.keys()) == list(sb.keys())
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_fp8_emulation_rounding_and_layer_choice():
    """The CPU emulation of the CVAE_FP8 path (checker for test_hip_parity's fp8 tests): OCP e4m3
    round-to-nearest-even with saturation, power-of-two weight scales with 4x headroom, and the
    layers that run in fp8 (padded K % 64 == 0)."""
    import numpy as np
    from oracle import cvae_np
    a = np.array([1.0625, 1.1875, 1.09375, 500.0, -1e4, 0.001, 2.0 ** -10, 240.0, 272.0], np.float32)
    np.testing.assert_array_equal(cvae_np.e4m3(a),
                                  [1.0, 1.25, 1.125, 448.0, -448.0, 2.0 ** -9, 0.0, 240.0, 256.0])
    assert cvae_np.f8_scale(np.array([0.05, -0.1], np.float32)) == 1024.0  # 2^floor(log2(448 / 0.4))
    torch_sd = OracleCVAE(100, 6, 8).state_dict()
    p = {k: v.numpy() for k, v in torch_sd.items()}
    f8 = cvae_np.fp8_layers(p, 100, 6, 8)
    # cfg2: K=600 (pad 608) and K=Z+H=136 (pad 160) and K=2 stay bf16; every 128/256-wide K is fp8
    assert set(f8) == {"condition_encoder.2", "encoder.3", "encoder.5", "encoder.7", "fc_mu", "fc_logvar",
                       "decoder.2", "decoder.4", "decoder.6"}
    assert f8["fc_mu"] == f8["fc_logvar"]
    p5 = {k: v.numpy() for k, v in OracleCVAE(200, 6, 512, 128, 8, 8).state_dict().items()}
    f85 = cvae_np.fp8_layers(p5, 200, 6, 512, 128, 8, 8)
    assert "encoder.1" in f85 and "decoder.0" in f85 and "condition_encoder.0" not in f85



def test_class_embedding_layout(cl):
    """BASELINE cfg4: the scenario-class embedding adds one parameter tensor, LAST (nn.Embedding
    layout), and widens fc (2H+E inputs) and decoder.0 (Z+H+E inputs); the reference's 24 keys
    keep their order."""
    from cvae_amd import ConditionalTrajectoryVAE, config_info
    n, nt, lds = config_info(10, 3, 8, 128, n_classes=4, class_dim=16)
    m = ConditionalTrajectoryVAE(10, 3, 8, n_classes=4, class_dim=16)
    ref = OracleCVAE(10, 3, 8, n_classes=4, class_dim=16)
    keys = list(m.state_dict().keys())
    assert keys == list(ref.state_dict().keys()) and nt == 25 == len(keys)
    assert keys[:24] == list(OracleCVAE(10, 3, 8).state_dict().keys())
    assert keys[-1] == "class_embedding.weight" and tuple(m.state_dict()[keys[-1]].shape) == (4, 16)
    assert n == sum(p.numel() for p in m.parameters()) and 0 < lds <= 160 * 1024
    assert m.fc_mu.weight.shape == (8, 2 * 128 + 16) and m.decoder[0].weight.shape == (128, 8 + 128 + 16)
    from cvae_amd._lib import CvaeError
    with pytest.raises(CvaeError, match="class_dim"):
        config_info(10, 3, 8, 128, n_classes=4, class_dim=6)
