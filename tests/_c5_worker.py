"""Worker of tests/test_gpu_multirank.py (one process per rank, launched by
torch.distributed.run; BGX_DIST_BACKEND=gloo lets 2 ranks share one GPU).

Runs PPOTrainer.iteration() (rollout on the rank's own game shard + the 4-epoch
update with the gradient all-reduce and the global return normalisation) and
checks, across ranks:
  * identical weights on every rank after the update;
  * global_normalize(R_rank) == the single-process (R - mean)/(std + 1e-5) over
    the concatenated returns of all ranks;
  * the distributed fp32 epoch == one single-process epoch over the
    concatenated batch (gradients averaged over equal shards = the full-batch mean).
Writes a JSON verdict per rank to $C5_OUT.<rank>.json."""
import copy
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]


def main():
    backend = os.environ.get("BGX_DIST_BACKEND", "gloo")
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    else:
        dist.init_process_group(backend)
    rank, ws = dist.get_rank(), dist.get_world_size()
    from bgx.train import PPOTrainer, lane_returns, ppo_epoch, features_and_masks
    from bgx.ppo import global_normalize
    out = {"rank": rank, "world_size": ws}
    B, T = 2048, 8
    tr = PPOTrainer(batch=B, horizon=T, seed=5, chunk=8192)
    # weights broadcast from rank 0 at construction
    flat0 = torch.cat([p.detach().reshape(-1) for p in tr.net.parameters()])
    g0 = [torch.empty_like(flat0) for _ in range(ws)]
    dist.all_gather(g0, flat0)
    out["init_identical"] = all(torch.equal(g0[0], g) for g in g0)
    # lanes differ across ranks (rank-offset dice seeds)
    rec0 = tr.eng.records()[:, :56].contiguous()
    gr = [torch.empty_like(rec0) for _ in range(ws)]
    dist.all_gather(gr, rec0)
    m = tr.iteration()
    out["episodes"] = m["episodes"]
    out["losses_finite"] = all(float(m[k]) == float(m[k]) for k in ("policy_loss", "value_loss", "entropy"))
    flat = torch.cat([p.detach().reshape(-1) for p in tr.net.parameters()])
    g1 = [torch.empty_like(flat) for _ in range(ws)]
    dist.all_gather(g1, flat)
    out["final_identical"] = all(torch.equal(g1[0], g) for g in g1)
    out["weights_moved"] = not torch.equal(flat, flat0)
    # global return normalisation vs the concatenated single-process formula
    R = lane_returns(tr.buf["rewards"], tr.buf["dones"]).reshape(-1)
    Rs = [torch.empty_like(R) for _ in range(ws)]
    dist.all_gather(Rs, R)
    full = torch.cat(Rs)
    ref = (full - full.mean()) / (full.std() + 1e-5)
    mine = global_normalize(R)
    out["norm_max_abs_err"] = float((mine - ref[rank * R.numel():(rank + 1) * R.numel()]).abs().max())
    # distributed fp32 epoch == single-process epoch over the concatenated batch
    recs = tr.buf["records"].reshape(-1, 64)
    acts, old = tr.buf["actions"].reshape(-1), tr.buf["logp"].reshape(-1)
    Rn = global_normalize(R)
    adv = Rn - tr.buf["values"].reshape(-1)
    N = recs.shape[0]
    net_d = copy.deepcopy(tr.net)
    opt_d = torch.optim.SGD(net_d.parameters(), lr=1.0)
    sc = torch.amp.GradScaler(device="cuda", enabled=False)
    ppo_epoch(net_d, opt_d, sc, [(*features_and_masks(recs, tr.A), acts, old, Rn, adv, recs)], N, 0.15, amp=False)
    pd = torch.cat([p.detach().reshape(-1) for p in net_d.parameters()])
    # gather every rank's batch and replay it as one process on rank 0
    def gather(x):
        xs = [torch.empty_like(x) for _ in range(ws)]
        dist.all_gather(xs, x.contiguous())
        return torch.cat(xs)
    R_all, recs_all, acts_all, old_all = gather(R), gather(recs), gather(acts), gather(old)
    vals_all = gather(tr.buf["values"].reshape(-1))
    if rank == 0:
        Rn_all = (R_all - R_all.mean()) / (R_all.std() + 1e-5)
        net_s = copy.deepcopy(tr.net)
        opt_s = torch.optim.SGD(net_s.parameters(), lr=1.0)
        f_all, l_all = features_and_masks(recs_all, tr.A)
        # world size 1 inside: a group holding only this rank
        solo = dist.new_group([0], backend="gloo")
        ppo_epoch(net_s, opt_s, sc, [(f_all, l_all, acts_all, old_all, Rn_all, Rn_all - vals_all, recs_all)],
                  N * ws, 0.15, group=solo, amp=False)
        ps = torch.cat([p.detach().reshape(-1) for p in net_s.parameters()])
        base = torch.cat([p.detach().reshape(-1) for p in tr.net.parameters()])
        du_d, du_s = pd - base, ps - base
        out["epoch_rel_err"] = float((du_d - du_s).norm() / du_s.norm())
    else:
        dist.new_group([0], backend="gloo")          # group creation is collective
    dist.barrier()
    with open(os.environ["C5_OUT"] + f".{rank}.json", "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
