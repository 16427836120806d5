"""First-light GPU check: run small configs on the GPU and compare with the CPU oracle.
Usage: python tools/gpu_debug.py [C1|C2|C3] [M] [R]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mrbo import configs  # noqa: E402
from mrbo.rollout import simulate_trajectory_mc_batch  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(name, M, R):
    pb = configs.problem(name, M=M, R=R)
    s = pb.surrogate
    n = s.observed
    osur = O.OracleSurrogate(s.X[:, :n], s.L[:n, :n], s.c[:n], s.y[:n], fmini=s.fmini())
    # primitives: eval_base at the restart points
    from mrbo.rollout import evaluate_base
    ev = evaluate_base(s, pb.x0s, [0.0])
    ob = O.eval_base(osur, pb.x0s)
    d = pb.cfg.d
    gmu = np.array([e.μ for e in ev])
    print(f"[{name}] eval_base mu maxrel", np.max(np.abs(gmu - ob[0]) / (np.abs(ob[0]) + 1e-300)),
          "sigma", np.max(np.abs(np.array([e.σ for e in ev]) - ob[1])),
          "alpha", np.max(np.abs(np.array([e.αxθ for e in ev]) - ob[2])),
          "H", np.max(np.abs(np.array([e.Hαx.ravel(order='F') for e in ev]).T - ob[3 + 3 * d:3 + 3 * d + d * d])))
    torch.cuda.synchronize()
    t = time.time()
    br = simulate_trajectory_mc_batch(pb.T, pb.tp, pb.x0s, pb.es.get_starts(), want_policy=True, want_obs=True)
    torch.cuda.synchronize()
    dt = time.time() - t
    g = br.numpy()
    print(f"[{name}] gpu {M*R} traj in {dt:.3f}s kernel {br.plan.last_kernel_ms():.2f} ms; status", np.unique(g["status"]),
          "evals mean", g["evals"][0].mean(), "value", g["evals"][1].mean(), "rich", g["evals"][2].mean(), "pairs", g["evals"][3].mean())
    t = time.time()
    o = O.simulate_mc(osur, pb.x0s, pb.tp.rnstream_sequence, pb.es.get_starts(), pb.lbs, pb.ubs, pb.cfg.h, nthreads=16)
    print(f"[{name}] oracle {time.time()-t:.2f}s status", np.unique(o["status"]), "evals mean", o["evals"].mean())
    same = np.all(np.abs(g["policy_x"] - o["policy_x"]) < 1e-6, axis=(0, 1))
    print(f"[{name}] policy agreement {same.mean():.4f}")
    dv = np.abs(g["values"] - o["values"])
    print(f"[{name}] values maxabs diff (all) {dv.max():.3e}; (agreeing) {dv[same].max() if same.any() else -1:.3e}")
    dg = np.abs(g["grad_x"] - o["grad_x"]).max(axis=0)
    print(f"[{name}] grad maxabs diff (agreeing) {dg[same].max() if same.any() else -1:.3e}")
    # replay mode: oracle with the GPU's policy points
    rp = np.asfortranarray(g["policy_x"][:, 1:, :, :])
    o2 = O.simulate_mc(osur, pb.x0s, pb.tp.rnstream_sequence, pb.es.get_starts(), pb.lbs, pb.ubs, pb.cfg.h,
                       replay_x=rp, nthreads=16)
    dv = np.abs(g["values"] - o2["values"])
    dg = np.abs(g["grad_x"] - o2["grad_x"])
    rel = dg / (np.abs(o2["grad_x"]) + 1e-12)
    print(f"[{name}] replay: values maxabs {dv.max():.3e}, grad maxabs {dg.max():.3e}, grad maxrel {rel.max():.3e}")
    print(f"[{name}] eto gpu {g['eto'][:4,0]} oracle {o['eto'][:4,0]}")


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    run(name, M, R)
