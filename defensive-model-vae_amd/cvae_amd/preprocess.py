"""Trajectory extraction from the simulator CSV logs: the step before training.

Restates ``Traj_Data_Process.py`` (the reference's dataset builder) with the same results, as
vectorised column operations instead of a per-row ``iterrows`` scan:

* ``SCENE_CONFIG`` (`Traj_Data_Process.py:8-25`): per scene, the row where the manoeuvre starts
  (first row whose start condition holds) and where it ends (first LATER row whose end
  condition holds; the trajectory stops before it);
* ``process_csv`` (`:72-122`): cut the ego (x, y) track between those rows, resample it to
  ``target_points`` points with ``np.linspace(..., dtype=int)`` indices (``point_mode``
  'normal', or 'extend_mid' = the midpoints between them), and prepend the time column
  ``k · time_interval · (n − 1)/(target_points − 1)``;
* ``collect_trajectories`` (`:125-141`), ``pad_and_save`` (`:144-150`): walk
  ``root/scene/action/*.csv`` in directory order and save the (N, target_points, 3) float64
  array ``TrajectoryDataset`` loads;
* ``generate_random_trajectories`` (`:31-69`): the 'random' mode, with the reference's
  ``random.uniform`` draw order (same outputs for the same ``random`` state).

The output files are the training inputs the reference ships (`training/DefensiveDataProcessed/
trajectory_sce{1..4}_cond.npy`); `tests/test_preprocess.py` checks them bit for bit.
"""
from __future__ import annotations

import os
import random

import numpy as np
import pandas as pd

ACTIONS = ["减速", "减速+转向", "转向"]  # decelerate, decelerate + steer, steer (Traj_Data_Process.py:27)


def _start_static(c):
    return (c["ego_y"] >= 18) & (c["sv2_vx"] != 0) & (c["sv2_vy"] != 0)


def _end_static(c):
    return c["ego_y"] >= 95


def _start_dynamic(c):
    return c["sv1_yaw"] < -170


def _end_dynamic(c):
    return c["ego_x"] < -186


def _start_predictable(c):
    return (c["sv1_vx"] != 0) & (c["sv1_vy"] != 0) & (c["ego_y"] <= 40) & (c["ego_y"] != 0)


def _end_predictable(c):
    return c["ego_y"] <= -80


def _start_unpredictable(c):
    return ((c["ego_x"] - c["sv1_x"]) ** 2 + (c["ego_y"] - c["sv1_y"]) ** 2 <= 40 ** 2) & (c["sv1_yaw"] >= -89.9)


def _end_unpredictable(c):
    return (c["sv1_x"] > 15) & (c["sv1_yaw"] < -85)


# scene → (start condition, end condition), each a vectorised predicate over the columns
# (Traj_Data_Process.py:8-25: the start predicate there is already vectorised; the end predicate
# is applied row by row in an iterrows loop, here over whole columns)
SCENE_CONFIG = {
    "StaticBlindTown05": (_start_static, _end_static),
    "DynamicBlindTown05": (_start_dynamic, _end_dynamic),
    "PredictableMovementTown05": (_start_predictable, _end_predictable),
    "UnpredictableMovementTown04": (_start_unpredictable, _end_unpredictable),
}

# columns the conditions and the track read
COLUMNS = ("ego_x", "ego_y", "sv1_x", "sv1_y", "sv1_vx", "sv1_vy", "sv1_yaw", "sv2_vx", "sv2_vy")


def _first_true(mask):
    idx = np.flatnonzero(np.asarray(mask, dtype=bool))
    return int(idx[0]) if idx.size else None


def process_frame(cols, scene, target_points=5, point_mode="normal", time_interval=0.015):
    """``process_csv`` on already-parsed columns (name → 1-D float64 array of the CSV's rows).

    Returns the (target_points, 3) array [time, ego_x, ego_y] or None (no start row, or fewer
    rows than ``target_points`` between start and end).
    """
    start_cond, end_cond = SCENE_CONFIG[scene]
    start = _first_true(start_cond(cols))                      # :76-83
    if start is None:
        return None
    rest = {k: np.asarray(v)[start + 1:] for k, v in cols.items()}
    end_rel = _first_true(end_cond(rest))                      # :87-93, rows after the start row
    stop = len(cols["ego_x"]) if end_rel is None else start + 1 + end_rel
    if "ego_x" not in cols or "ego_y" not in cols:
        return None
    traj = np.stack([np.asarray(cols["ego_x"])[start:stop], np.asarray(cols["ego_y"])[start:stop]], axis=1)
    n = len(traj)
    if n < target_points:                                      # :101-102
        return None
    indices = np.linspace(0, n - 1, target_points, dtype=int)  # :105
    if point_mode == "normal":
        traj = traj[indices]
    elif point_mode == "extend_mid":                           # :109-114
        mid = np.ceil((indices[:-1] + indices[1:]) / 2).astype(int)
        traj = traj[np.append(np.insert(mid[:-1], 0, indices[0]), indices[-1])]
    times = np.arange(target_points) * time_interval * ((n - 1) / (target_points - 1))  # :117
    return np.column_stack((times, traj))


def read_columns(csv_path):
    """The columns ``process_frame`` needs, parsed exactly as the reference parses the file
    (``pandas.read_csv`` defaults)."""
    df = pd.read_csv(csv_path, usecols=lambda c: c in COLUMNS)  # same parser, fewer columns
    return {k: df[k].to_numpy() for k in COLUMNS if k in df.columns}


def process_csv(csv_path, scene, action=None, target_points=5, point_mode="normal", time_interval=0.015):
    """Traj_Data_Process.process_csv (`:72-122`); ``action`` is unused there too."""
    return process_frame(read_columns(csv_path), scene, target_points, point_mode, time_interval)


# scene → (id of the device kernel's predicate pair, columns its predicates read)
_SCENE_ID = {
    "StaticBlindTown05": (0, ("ego_y", "sv2_vx", "sv2_vy")),
    "DynamicBlindTown05": (1, ("sv1_yaw", "ego_x")),
    "PredictableMovementTown05": (2, ("sv1_vx", "sv1_vy", "ego_y")),
    "UnpredictableMovementTown04": (3, ("ego_x", "sv1_x", "ego_y", "sv1_y", "sv1_yaw")),
}


def process_frames_device(frames, scene, target_points=5, point_mode="normal", time_interval=0.015,
                          device="cuda"):
    """``process_frame`` for many parsed CSVs in ONE launch of the HIP extraction kernel
    (csrc/cvae_extract.h; C-ABI ``cvae_extract_trajectories``): the columns of all files are
    stacked into one float64 [9][rows] device array, one workgroup per file finds the start row
    and the end row, resamples the track and forms the time column.  Same results as
    ``process_frame`` bit for bit (list of (target_points, 3) arrays or None, in input order).
    Fails loudly without the HIP extension (no host fallback)."""
    import ctypes as C
    import torch
    from ._lib import check, lib
    if point_mode not in ("normal", "extend_mid"):
        raise ValueError(f"unknown point_mode {point_mode!r}")
    if target_points < 2:
        raise ValueError("target_points must be >= 2")
    sid, needed = _SCENE_ID[scene]
    lens, usable = [], []
    for cols in frames:
        for k in needed:  # the host predicates raise KeyError on a missing column: so do we
            if k not in cols:
                raise KeyError(k)
        n = len(next(iter(cols.values()))) if cols else 0
        lens.append(n)
        usable.append("ego_x" in cols and "ego_y" in cols)
    n_rows = int(sum(lens))
    host = np.zeros((len(COLUMNS), n_rows), np.float64)
    r = 0
    for cols, n in zip(frames, lens):
        for c, name in enumerate(COLUMNS):
            if name in cols:
                host[c, r:r + n] = np.asarray(cols[name], dtype=np.float64)
        r += n
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    dev = torch.device(device)
    d_cols = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_out = torch.empty((len(frames), target_points, 3), dtype=torch.float64, device=dev)
    d_valid = torch.empty(len(frames), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    check(lib().cvae_extract_trajectories(C.c_void_p(d_cols.data_ptr()), n_rows, C.c_void_p(d_off.data_ptr()),
                                          len(frames), sid, int(target_points), int(point_mode == "extend_mid"),
                                          float(time_interval), C.c_void_p(d_out.data_ptr()),
                                          C.c_void_p(d_valid.data_ptr()), C.c_void_p(stream)),
          "cvae_extract_trajectories")
    out, valid = d_out.cpu().numpy(), d_valid.cpu().numpy()
    return [out[f] if valid[f] and usable[f] else None for f in range(len(frames))]


def _scene_files(data_root, scene, actions):
    for action in actions:
        path = os.path.join(data_root, scene, action)
        if not os.path.exists(path):
            continue
        for fname in os.listdir(path):
            if fname.endswith(".csv"):
                yield action, os.path.join(path, fname)


def collect_trajectories(data_root, scenes, actions, target_points=5, point_mode="normal", time_interval=0.015,
                         device=None):
    """Traj_Data_Process.collect_trajectories (`:125-141`): every CSV under root/scene/action, in
    ``os.listdir`` order; trajectories that fail extraction are skipped.  ``device`` (e.g.
    "cuda"): parse on the host, extract every file of a scene in one kernel launch
    (``process_frames_device``)."""
    out = []
    for scene in scenes:
        files = list(_scene_files(data_root, scene, actions))
        if device is not None:
            ts = process_frames_device([read_columns(p) for _, p in files], scene, target_points, point_mode,
                                       time_interval, device)
        else:
            ts = (process_csv(p, scene, a, target_points, point_mode, time_interval) for a, p in files)
        out.extend(t for t in ts if t is not None and len(t) == target_points)
    return out


def pad_and_save(trajs, save_path):
    """Traj_Data_Process.pad_and_save (`:144-150`): (N, target_points, 3) float64 .npy."""
    arr = np.array(trajs)
    np.save(save_path, arr)
    return arr


def generate_random_trajectories(num_trajs, traj_length, max_angle_deviation=5.0, rng=None):
    """Traj_Data_Process.generate_random_trajectories (`:31-69`): unit-step random walks from the
    origin whose heading changes by U(−max, +max) degrees per step; (num_trajs, traj_length, 2).
    ``rng``: a ``random.Random`` (default: the module-level ``random`` state, as the reference)."""
    uni = (rng or random).uniform
    a_max = np.radians(max_angle_deviation)
    out = np.zeros((num_trajs, traj_length, 2))
    for n in range(num_trajs):
        ang = 0.0
        for i in range(1, traj_length):
            ang += uni(-a_max, a_max)
            out[n, i, 0] = out[n, i - 1, 0] + 1.0 * np.cos(ang)
            out[n, i, 1] = out[n, i - 1, 1] + 1.0 * np.sin(ang)
    return out


def main(argv=None):
    """``python -m cvae_amd.preprocess --root DefensiveData --scene StaticBlindTown05 --points 10
    --interval 0.02 --out trajectory_sce1_cond.npy`` (the reference's __main__ 'dataset' mode,
    Traj_Data_Process.py:153-186, with its parameters as flags)."""
    import argparse
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("--root", required=True)
    ap.add_argument("--scene", action="append", required=True, choices=sorted(SCENE_CONFIG))
    ap.add_argument("--action", action="append", default=None)
    ap.add_argument("--points", type=int, default=10)
    ap.add_argument("--interval", type=float, default=0.02)
    ap.add_argument("--mode", default="normal", choices=["normal", "extend_mid"])
    ap.add_argument("--out", required=True)
    ap.add_argument("--device", default=None, help="e.g. cuda: extract on the GPU (one launch per scene)")
    a = ap.parse_args(argv)
    trajs = collect_trajectories(a.root, a.scene, a.action or ACTIONS, a.points, a.mode, a.interval, a.device)
    if not trajs:
        raise SystemExit("no trajectory extracted")
    arr = pad_and_save(trajs, a.out)
    print(f"saved {arr.shape[0]} trajectories of {arr.shape[1]} points to {a.out}")


if __name__ == "__main__":
    main()
