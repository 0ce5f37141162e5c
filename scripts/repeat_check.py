"""Run-to-run repeatability of a training chain (GPU box): N forward_backward calls on the same
input must give the same loss and gradient bits.  A register hazard in the chain (a load that
overwrites an operand an in-flight MFMA has not read yet; an asm store whose data registers the
compiler reuses) shows up as a few calls whose bits differ.

  python3 scripts/repeat_check.py --workload wide --dtype fp8 --calls 200 [--batch 1024]

Prints one JSON line: calls, mismatching calls, the largest gradient difference.  CVAE_LIB selects
another build of the library (scripts/build_diag.sh)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "defensive-model-vae_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="wide", choices=["wide", "cfg2"])
    ap.add_argument("--dtype", default="fp8")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--calls", type=int, default=200)
    args = ap.parse_args()
    from cvae_amd import ConditionalTrajectoryVAE
    S, D, Z, NE, ND = (200, 6, 512, 8, 8) if args.workload == "wide" else (100, 6, 8, 4, 4)
    torch.manual_seed(0)
    m = ConditionalTrajectoryVAE(S, D, Z, 128, NE, ND)
    eng = m.attach(dtype=args.dtype, max_batch=args.batch, device="cuda:0")
    x = eng.as_input(torch.randn(args.batch, S, D, generator=torch.Generator().manual_seed(3)))
    eps = torch.randn(args.batch, Z, generator=torch.Generator().manual_seed(4)).cuda()
    l0 = eng.forward_backward(x, eps=eps).clone()
    g0 = eng.grads.clone()
    bad, worst = 0, 0.0
    for _ in range(args.calls):
        l = eng.forward_backward(x, eps=eps)
        if not (torch.equal(l, l0) and torch.equal(eng.grads, g0)):
            bad += 1
            worst = max(worst, float((eng.grads - g0).abs().max()))
    torch.cuda.synchronize()
    print(json.dumps({"workload": args.workload, "dtype": args.dtype, "batch": args.batch, "calls": args.calls,
                      "kernel": eng.train_kernel, "mismatching_calls": bad, "max_grad_diff": worst,
                      "lib": os.environ.get("CVAE_LIB", "default")}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
