"""Subprocess body of tests/test_gpu_dp.py::test_rccl_world1_graph_cache_matches_eager
(a separate process: it owns an RCCL process group).

BASELINE config 4 with VoiceBank-style padding at world size 1 over RCCL: a
bf16 HybridViT with dropout trained through GraphedTrainStep WITH a
GradAllReducer (bucket all-reduces from the grad hooks, a sliced pos_embed)
on batches of three different T (LRU cap 2: a shape's graph is evicted and
captured again), against an identical copy stepped eagerly with its own
reducer from the same dropout seed state.  Prints one JSON line: whether every
step's parameters and loss matched bit for bit, and the cache counters."""

import copy
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KW = dict(encoder_channels=[8, 16, 32], embed_dim=128, num_heads=2, num_layers=2, decoder_channels=[32, 16, 8, 1],
          precision="bf16")


def main():
    port = int(sys.argv[1])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    import importlib

    import hvit_amd_loader

    hv = hvit_amd_loader.load()
    from hvit_amd.dp import GradAllReducer

    ts = importlib.import_module("hvit_amd.train_step")
    torch.manual_seed(0)
    ma = hv.HybridViT(**KW).cuda().train()
    mb = copy.deepcopy(ma)
    ra = GradAllReducer(ma, bucket_mb=1.0, sliced={"pos_encoding.pos_embed": 64})
    rb = GradAllReducer(mb, bucket_mb=1.0, sliced={"pos_encoding.pos_embed": 64})
    oa = hv.FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    ob = hv.FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    crit = hv.CombinedLoss()
    step = ts.GraphedTrainStep(ma, crit, oa, reducer=ra, max_graphs=2, warmup=1)
    ma.set_dropout_state(2024)
    mb.set_dropout_state(2024)
    g = torch.Generator().manual_seed(8)
    Ts = [64, 64, 64, 48, 48, 48, 80, 80, 64, 64, 48, 48]
    bad = []
    for i, T in enumerate(Ts):
        x = torch.rand(2, 1, 48, T, generator=g).cuda()
        t = torch.rand(2, 1, 48, T, generator=g).cuda()
        la = step(x, t)
        lb = crit(mb(x), t)
        lb.backward()
        rb.finish()
        ob.step()
        ob.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        same = la.item() == lb.item() and all(torch.equal(pa.detach(), pb.detach())
                                              for pa, pb in zip(ma.parameters(), mb.parameters()))
        if not same:
            bad.append((i, T))
    print(json.dumps({"bad": bad, "captures": step.captures, "replays": step.replays, "cached": len(step.cache),
                      "dropout_state_equal": bool(torch.equal(ma.dropout_state(), mb.dropout_state()))}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
