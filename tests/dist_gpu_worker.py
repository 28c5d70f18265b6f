"""Worker of tests/test_dist_gpu.py (not collected by pytest): one rank of a world-N run of
the sharded MaxK aggregation on the one GPU of the box -- HIP kernels on cuda:0, gloo
collectives staged through host memory (N processes share the device, so each keeps one HIP
hardware queue: tools/share_probe.py).  Reads the graph and features the parent wrote, runs
forward + backward through maxk_dist in both exchange modes and writes its rows back.

    python tests/dist_gpu_worker.py DIR RANK WORLD PORT [BACKEND]

BACKEND "nccl" (RCCL): one GPU per rank (cuda:RANK), collectives on device over xGMI; only
where at least WORLD GPUs are visible (tests/test_dist_gpu.py skips it otherwise).
"""
import os
import sys

BACKEND = sys.argv[5] if len(sys.argv) > 5 else "gloo"
if BACKEND == "gloo":
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")  # ranks share one device; before HIP starts

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_dist  # noqa: E402


def main(d, rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    if BACKEND == "nccl":
        dev = torch.device("cuda", rank)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    with np.load(os.path.join(d, "graph.npz"), allow_pickle=False) as z:
        g = {n: z[n] for n in z.files}
    k, D = int(g["k"]), int(g["D"])
    to = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    row_ptr, col, val = to(g["row_ptr"]), to(g["col"]), to(g["val"])
    deg = to(g["deg"])
    out = {}
    for mode in ("gather", "halo"):
        shard = maxk_dist.ShardedMaxK(row_ptr, col, val, rank, world, device=dev, mode=mode)
        v0, v1 = shard.v0, shard.v1
        tv, ti = mk.topk_cbsr(to(g["x"][v0:v1]), k)
        tv.requires_grad_(True)
        y = maxk_dist.sharded_maxk_spgemm(shard, tv, ti, D, deg[v0:v1])
        y.backward(to(g["g"][v0:v1]))
        torch.cuda.synchronize()
        out[f"{mode}_y"] = y.detach().cpu().numpy()
        out[f"{mode}_gs"] = tv.grad.cpu().numpy()
        out[f"{mode}_bounds"] = np.array(shard.bounds, np.int64)
        out[f"{mode}_fwd_recv"] = np.int64(shard.exchange_bytes(k)["fwd_recv"])
    np.savez(os.path.join(d, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
