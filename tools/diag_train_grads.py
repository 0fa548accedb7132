"""Per-parameter gradient error of a training fixture (diagnostic, GPU): for each parameter, max |grad -
ref| / max |ref| and the worst elements.  Usage: python tools/diag_train_grads.py NAME [mlp]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import test_gpu_train as T  # noqa: E402


def main():
    name = sys.argv[1]
    mlp = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    g, tr, sk, out, loss = T._run(name, mlp)
    rows = []
    for net_name, net in (("fn", tr.network_fn), ("fine", tr.network_fine)):
        for pname, p in net.named_parameters():
            key = f"grad_{net_name}__{pname}"
            if not g.has(key) or p.grad is None:
                continue
            a = p.grad.detach().cpu().numpy().reshape(-1)
            if g.has(key + "__idx"):
                a = a[g[key + "__idx"]]
            ref = g[key]
            d = np.abs(a - ref)
            rows.append((float(d.max() / max(np.abs(ref).max(), 1e-30)), key, float(d.max()), float(np.abs(ref).max()),
                         np.argsort(-d)[:4].tolist(), a[np.argsort(-d)[:4]].tolist(), ref[np.argsort(-d)[:4]].tolist()))
    rows.sort(reverse=True)
    for r in rows[:12]:
        print(f"{r[0]:.3e}  {r[1]}  max|d| {r[2]:.3e} max|ref| {r[3]:.3e}  idx {r[4]}  gpu {np.round(r[5], 7)}  ref {np.round(r[6], 7)}")
    gs = sk.grad.detach().cpu().numpy()
    print("dL/dskts", float(np.abs(gs - g["grad_skts"]).max() / np.abs(g["grad_skts"]).max()))


if __name__ == "__main__":
    main()
