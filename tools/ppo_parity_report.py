"""Print the measured margins of the PPO-update parity tests (GPU): the trainer's
update vs golden G6b (fp32) / G6c (fp16), and the fused fp16 epoch vs the fp32
torch epoch at 2^21 rows with the per-row gradient scale of bgx.train (REF_ROWS)
and with the old scale / n (REF_ROWS = inf)."""
import copy
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"), os.path.join(ROOT, "tests")]

import bgx.train as T  # noqa: E402
from bgx.engine import encode  # noqa: E402
from bgx.ppo import global_normalize  # noqa: E402
from test_gpu_train import _records_from_fixture  # noqa: E402


def golden_margins():
    out = {}
    for v in ("fp32", "fp16"):
        g = dict(np.load(os.path.join(ROOT, "tests", "golden", f"ppo_{v}.npz")))
        tr = T.PPOTrainer(batch=int(g["N"]), horizon=int(g["T"]), returns="reference", amp=(v == "fp16"))
        tr.net.load_state_dict({k[5:]: torch.from_numpy(x) for k, x in g.items() if k.startswith("init_")})
        rec = _records_from_fixture(g).cuda()
        tr.load_rollout(rec, torch.from_numpy(g["actions"]), torch.from_numpy(g["old_logp"]),
                        torch.from_numpy(g["old_v"]), torch.from_numpy(g["rewards"]), torch.from_numpy(g["dones"]))
        m = tr.update()
        got = np.array([m["policy_loss"], m["value_loss"], m["entropy"], m["total_loss"]])
        w = {}
        for k, x in tr.net.state_dict().items():
            du = x.cpu().numpy() - g["init_" + k]
            dr = g["final_" + k] - g["init_" + k]
            w[k] = {"max_abs": float(np.abs(du - dr).max()), "frac_gt_1e-4": float(np.mean(np.abs(du - dr) > 1e-4)),
                    "max_update": float(np.abs(dr).max())}
        out[v] = {"loss_max_abs": float(np.abs(got - g["losses"]).max()), "weights": w}
    return out


def large_batch(ref_rows):
    T.REF_ROWS = ref_rows
    torch.manual_seed(0)
    tr = T.PPOTrainer(batch=65536, horizon=32, seed=9)
    tr.rollout()
    buf = tr.buf
    R = global_normalize(T.lane_returns(buf["rewards"], buf["dones"]).reshape(-1))
    adv = R - buf["values"].reshape(-1)
    recs = buf["records"].reshape(-1, 64)
    acts, old = buf["actions"].reshape(-1), buf["logp"].reshape(-1)
    N = recs.shape[0]

    def chunks(with_legal):
        for s in range(0, N, 1 << 19):
            f, legal = T.features_and_masks(recs[s:s + (1 << 19)], tr.A)
            yield f, legal if with_legal else None, acts[s:s + (1 << 19)], old[s:s + (1 << 19)], \
                R[s:s + (1 << 19)], adv[s:s + (1 << 19)], recs[s:s + (1 << 19)]
    res = {}
    for amp in (False, True):
        net = copy.deepcopy(tr.net)
        sc = torch.amp.GradScaler(device="cuda")
        T.ppo_epoch(net, torch.optim.Adam(net.parameters()), sc, chunks(not amp), N, 0.15, amp=amp, fused=amp,
                    step=False)
        res[amp] = [p.grad.detach().float() / sc.get_scale() for p in net.parameters()]
    return {n: float(((a - b).norm() / a.norm()).item())
            for (n, _), a, b in zip(tr.net.named_parameters(), res[False], res[True])}


if __name__ == "__main__":
    rep = {"golden": golden_margins(), "large_batch_rel_err": large_batch(4096),
           "large_batch_rel_err_scale_over_n": large_batch(float("inf"))}
    print(json.dumps(rep, indent=1))
