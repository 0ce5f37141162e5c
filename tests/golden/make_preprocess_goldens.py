"""Fixtures for tests/test_preprocess.py (run here, where /root/reference exists):

* for two CSV logs per scene of the reference's DefensiveData, the columns the scene conditions
  and the ego track read (float64, as pandas parses them) and the reference's own
  ``Traj_Data_Process.process_csv`` output for three parameter sets;
* a full check of every CSV under DefensiveData against the reference (recorded counts), and of
  ``collect_trajectories`` against the shipped ``trajectory_sce{1,2,3}_cond.npy`` (same set of
  trajectories; the order is ``os.listdir`` order on the author's machine).

    python tests/golden/make_preprocess_goldens.py
"""
import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "defensive-model-vae_amd"), "/root/reference"]
import Traj_Data_Process as R  # noqa: E402  (the reference, imported read-only)
from cvae_amd import preprocess as P  # noqa: E402

DATA = "/root/reference/DefensiveData"
PARAMS = [(10, "normal", 0.02), (5, "extend_mid", 0.015), (12, "normal", 0.025)]


def ref_process(path, scene, action, tp, mode, ti):
    with contextlib.redirect_stdout(io.StringIO()):
        return R.process_csv(path, scene, action, tp, mode, ti)


def main():
    out = {}
    meta = {"params": PARAMS, "files": []}
    checked = mism = 0
    for scene in P.SCENE_CONFIG:
        picked = 0
        for action in P.ACTIONS:
            d = os.path.join(DATA, scene, action)
            if not os.path.exists(d):
                continue
            for f in sorted(os.listdir(d)):
                if not f.endswith(".csv"):
                    continue
                path = os.path.join(d, f)
                for tp, mode, ti in PARAMS:
                    r = ref_process(path, scene, action, tp, mode, ti)
                    o = P.process_csv(path, scene, action, tp, mode, ti)
                    checked += 1
                    mism += int((r is None) != (o is None) or (r is not None and not np.array_equal(r, o)))
                if picked < 2:
                    k = len(meta["files"])
                    cols = P.read_columns(path)
                    for c, v in cols.items():
                        out[f"f{k}/{c}"] = v
                    for j, (tp, mode, ti) in enumerate(PARAMS):
                        r = ref_process(path, scene, action, tp, mode, ti)
                        out[f"f{k}/out{j}"] = r if r is not None else np.zeros((0, 3))
                    meta["files"].append({"scene": scene, "action": action, "name": f})
                    picked += 1
    shipped = {}
    for sce, scene, ti in ((1, "StaticBlindTown05", 0.02), (2, "DynamicBlindTown05", 0.025),
                           (3, "PredictableMovementTown05", 0.015)):
        ours = np.array(P.collect_trajectories(DATA, [scene], P.ACTIONS, 10, "normal", ti))
        ref = np.load(f"/root/reference/training/DefensiveDataProcessed/trajectory_sce{sce}_cond.npy")
        key = lambda a: a[np.lexsort(a[:, :, 1:].reshape(len(a), -1).T[::-1])]  # noqa: E731
        shipped[f"sce{sce}"] = bool(ours.shape == ref.shape and np.array_equal(key(ours), key(ref)))
    import random
    random.seed(7)
    out["random_walks"] = R.generate_random_trajectories(5, 20, 5.0)  # random.seed(7) stream
    meta["all_csv_checked"] = checked
    meta["all_csv_mismatches"] = mism
    meta["shipped_npy_equal_as_sets"] = shipped
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "preprocess.npz"), **out)
    print(json.dumps({k: v for k, v in meta.items() if k != "files"}), len(meta["files"]), "files stored")


if __name__ == "__main__":
    main()
