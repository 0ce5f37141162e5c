"""SURVEY §8f-3 on the GPU: the HIP extraction kernel (C-ABI cvae_extract_trajectories, via
cvae_amd.preprocess.process_frames_device) against the reference's own Traj_Data_Process outputs
(tests/golden/preprocess.npz) and against the host restatement on adversarial synthetic logs
(predicate boundaries, no start, no end, ragged and empty files, long files).  Bit-exact: float64."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "defensive-model-vae_amd"))
from cvae_amd import preprocess as P  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden", "preprocess.npz")


def _same(got, want):
    if want is None or (hasattr(want, "size") and want.size == 0):
        return got is None
    return got is not None and got.dtype == np.float64 and np.array_equal(got, want)


def test_device_extraction_matches_reference_goldens():
    d = np.load(GOLD)
    meta = json.loads(bytes(d["meta"]).decode())
    for scene in P.SCENE_CONFIG:
        ks = [k for k, f in enumerate(meta["files"]) if f["scene"] == scene]
        frames = [{c: d[f"f{k}/{c}"] for c in P.COLUMNS if f"f{k}/{c}" in d} for k in ks]
        for j, (tp, mode, ti) in enumerate(meta["params"]):
            got = P.process_frames_device(frames, scene, tp, mode, ti)
            for k, g in zip(ks, got):
                assert _same(g, d[f"f{k}/out{j}"]), (scene, k, tp, mode)


def _pick(rng, n, common, rare, p_rare=0.03):
    """Mostly ``common`` values, with predicate-boundary ``rare`` values at rate ``p_rare``."""
    v = rng.choice(common, n)
    hit = rng.random(n) < p_rare
    v[hit] = rng.choice(rare, int(hit.sum()))
    return v


def _synthetic(rng, n, scene):
    """A log whose columns sit on and around the scene's predicate thresholds."""
    c = {k: rng.choice([0.0, 1.0, -1.0, 2.5], n) for k in P.COLUMNS}
    c["ego_y"] = _pick(rng, n, [0.0, 17.999999999999996, 18.0, 40.0, 40.00000000000001, 30.0, 60.0],
                       [95.0, 94.99999999999999, -80.0, -79.99999999999999])
    c["ego_x"] = _pick(rng, n, [-100.0, 10.0, 0.0, -185.99999999999997], [-186.0, -186.00000000000003])
    c["sv1_yaw"] = _pick(rng, n, [-170.0, -170.00000000000003, -89.9, -89.90000000000001, 0.0, -84.9],
                         [-85.00000000000001, -85.0])
    c["sv1_x"] = _pick(rng, n, [15.0, 0.0, 10.0], [15.000000000000002, 40.0])
    c["sv1_y"] = rng.choice([0.0, 40.0, 24.0, 32.0], n)
    if scene == "UnpredictableMovementTown04":  # exact distance-40 hits: (ego - sv1) = (24, 32)
        c["ego_x"] = c["sv1_x"] + rng.choice([24.0, 24.000000000000004, 0.0, 50.0], n)
        c["ego_y"] = c["sv1_y"] + rng.choice([32.0, 31.999999999999996, 0.0], n)
    c["sv1_vx"][rng.random(n) < 0.02] = np.nan
    return c


@pytest.mark.parametrize("scene", sorted(P.SCENE_CONFIG))
def test_device_extraction_matches_host_on_boundaries(scene):
    rng = np.random.default_rng(sum(map(ord, scene)))
    lens = [0, 1, 2, 5, 6, 7, 33, 255, 256, 257, 1000, 40000] + list(rng.integers(3, 3000, 40))
    frames = [_synthetic(rng, int(n), scene) for n in lens]
    for tp, mode, ti in [(5, "normal", 0.015), (10, "extend_mid", 0.02), (2, "normal", 0.025), (37, "extend_mid", 0.1)]:
        got = P.process_frames_device(frames, scene, tp, mode, ti)
        n_valid = 0
        for f, g in zip(frames, got):
            want = P.process_frame(f, scene, tp, mode, ti)
            assert _same(g, want), (scene, len(f["ego_x"]), tp, mode)
            n_valid += want is not None
        assert n_valid > 5  # the cases exercise the resampling, not only the None paths


def test_device_extraction_rejects_bad_arguments():
    frames = [{k: np.zeros(8) for k in P.COLUMNS}]
    with pytest.raises(ValueError):
        P.process_frames_device(frames, "StaticBlindTown05", 1)
    with pytest.raises(KeyError):
        P.process_frames_device([{"ego_x": np.zeros(3)}], "StaticBlindTown05", 2)
    assert P.process_frames_device([], "StaticBlindTown05", 5) == []
