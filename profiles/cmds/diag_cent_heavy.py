"""Diagnostics of the heaviest centralised searches (n = 10, N = 5 by default): solves the given
seeds' t = 0 platoons (bench.py --controller cent inputs) alone, with a QP cap, and prints per
platoon the status, QPs and time.  With HVP_CENT_DEBUG=6 the library prints QPs per search depth.

    python profiles/cmds/diag_cent_heavy.py --seeds 123 456 --max-nodes 20000000
    python profiles/cmds/diag_cent_heavy.py --from-bench gpurun_out/x.jsonl --top 2
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hybrid-vehicle-platoon_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="*", default=[])
    ap.add_argument("--from-bench", default=None)
    ap.add_argument("--top", type=int, default=1)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--N", type=int, default=5)
    ap.add_argument("--max-nodes", type=int, default=2_000_000)
    ap.add_argument("--save", default=None, help="npz of the platoons' x0 (for the oracle)")
    a = ap.parse_args()
    seeds = list(a.seeds)
    if a.from_bench:
        for line in open(a.from_bench):
            if line.strip().startswith("{"):
                seeds += [h[0] for h in json.loads(line)["heaviest"][:a.top]]
    import torch

    from hvp import tables
    from hvp.cent import CentSolver, cent_problem
    from hvp.env import derive_env_seed, initial_platoon_state
    from hvp.models import PwaGearVehicle

    n, N = a.n, a.N
    veh = PwaGearVehicle(800)
    system = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    x0 = np.stack([initial_platoon_state(n, derive_env_seed(int(s))).reshape(n, 2).astype(np.float64) for s in seeds])
    if a.save:
        np.savez(a.save, seeds=np.array(seeds), x0=x0)
    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    dev = torch.device("cuda", 0)
    sv = CentSolver(cent_problem(N), [system], device=0)
    for j, s in enumerate(seeds):
        ts = torch.zeros((1, n), dtype=torch.int32, device=dev)
        tx = torch.from_numpy(x0[j:j + 1]).to(dev)
        tl = torch.from_numpy(lead[None].copy()).to(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = sv.solve_device(ts, tx, tl, max_nodes=a.max_nodes)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"seed": int(s), "status": int(o["status"][0]), "nodes": int(o["nodes"][0]),
                          "iters": int(o["iters"][0]), "cost": float(o["cost"][0]), "s": dt,
                          "x0": x0[j].tolist(),
                          "regions": o["region"][0].cpu().numpy().tolist()}), flush=True)


if __name__ == "__main__":
    main()
