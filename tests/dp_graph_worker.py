"""Subprocess body of tests/test_gpu_dp.py::test_rccl_world1_dp_graph_matches_eager
(a separate process: it owns an RCCL process group).

BASELINE config 4's step as bench.py runs it, at world size 1 over RCCL: a
bf16 HybridViT train step with dropout, GradAllReducer (bucket all-reduces
launched from the grad hooks), FusedAdamW(capturable) -- captured once in a
hipGraph and replayed, against an identical copy stepped eagerly from the same
dropout seed state.  Prints one JSON line: per-replay max relative parameter
difference, loss pairs, and whether the graph's gradients were reduced in the
bucket buffers."""

import copy
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (D = 256 and 64 tokens per sample: the ViT weight gradients take the grouped launch, so the DP buckets
# holding them are deferred until its flush -- one grouped launch per step, checked below)
KW = dict(encoder_channels=[8, 16, 32], embed_dim=256, num_heads=4, num_layers=2, decoder_channels=[32, 16, 8, 1],
          precision="bf16")


def main():
    port = int(sys.argv[1])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    import hvit_amd_loader

    hv = hvit_amd_loader.load()
    from hvit_amd.dp import GradAllReducer

    torch.manual_seed(0)
    ma = hv.HybridViT(**KW).cuda().train()
    mb = copy.deepcopy(ma)
    ra = GradAllReducer(ma, bucket_mb=1.0, sliced={"pos_encoding.pos_embed": 64})
    rb = GradAllReducer(mb, bucket_mb=1.0, sliced={"pos_encoding.pos_embed": 64})
    oa = hv.FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    ob = hv.FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    crit = hv.CombinedLoss()
    g = torch.Generator().manual_seed(4)
    x = torch.rand(2, 1, 128, 128, generator=g).cuda()
    t = torch.rand(2, 1, 128, 128, generator=g).cuda()

    def step(m, r, o):
        loss = crit(m(x), t)
        loss.backward()
        r.finish()
        o.step()
        o.zero_grad(set_to_none=True)
        return loss

    ma.set_dropout_state(777)
    mb.set_dropout_state(777)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        HF = sys.modules["hvit_amd.functional"]
        n0 = HF.WG_LAUNCHES
        for _ in range(2):
            step(ma, ra, oa)
        group_launches = (HF.WG_LAUNCHES - n0) / 2
    torch.cuda.current_stream().wait_stream(side)
    from hvit_amd.dp import quiesce_for_capture
    quiesce_for_capture()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):  # (the watchdog thread polls events)
        static_loss = step(ma, ra, oa)
    for _ in range(2):
        step(mb, rb, ob)
    rel, losses = [], []
    for _ in range(3):
        graph.replay()
        lb = step(mb, rb, ob)
        torch.cuda.synchronize()
        losses.append((static_loss.item(), lb.item()))
        rel.append(max(((pa.detach() - pb.detach()).abs().max() / pb.detach().abs().max().clamp_min(1e-30)).item()
                       for pa, pb in zip(ma.parameters(), mb.parameters())))
    exact = all(torch.equal(pa.detach(), pb.detach()) for pa, pb in zip(ma.parameters(), mb.parameters()))
    print(json.dumps({"rel": rel, "losses": losses, "exact": exact, "group_launches_per_step": group_launches,
                      "steps": float(oa.state[next(ma.parameters())]["step"]),
                      "dropout_state_equal": bool(torch.equal(ma.dropout_state(), mb.dropout_state()))}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
