"""Accumulator batch size sweep (round 5): B simple-example proofs (BN254,
k = 17) from their serialized bytes through pm_accum_batch_proofs_device, for
B in $BS (default 16 .. 4096), one JSON line per B with the wall time per
batch and the per-kernel times (HIP events around every launch, a separate
set of steps).  Feeds the config-5 projection (BASELINE configs[4]: 256
proofs over 8 GPUs = 32 per rank) and the large-batch throughput rows of
DESIGN.md.  Usage: python tools/accum_scaling.py > out.jsonl"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd")]
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402
import workloads as Wk  # noqa: E402

KERNELS = ("proof_decode", "transcript", "acc_ladder", "acc_scalars", "acc_termmul", "acc_sum")


def main():
    bs = [int(x) for x in os.environ.get("BS", "16,32,64,128,256,512,1024,2048,4096").split(",")]
    logn, reps = int(os.environ.get("LOGN", "17")), int(os.environ.get("REPS", "20"))
    ctx = H.Context(0)
    if os.environ.get("LADDER"):  # force the chain form (pm_ctx_set_accum_ladder)
        ctx.set_accum_ladder(int(os.environ["LADDER"]))
    if os.environ.get("TWIST"):  # pm_ctx_set_accum_option(PM_ACC_OPT_TWIST, v)
        ctx.set_accum_option(H.ACC_OPT_TWIST, int(os.environ["TWIST"]))
    if os.environ.get("SPLIT"):  # lanes per term of the split form, log2 (pm_ctx_set_accum_split)
        ctx.set_accum_split(int(os.environ["SPLIT"]))
    shape = Wk.simple_example_shape(ctx, H.BN254, logn)
    for B in bs:
        batch = Wk.SyntheticBatch(ctx, shape, B)
        batch.to_proof_bytes(shape)
        for _ in range(3):
            batch.run_bytes(ctx, shape)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            batch.run_bytes(ctx, shape)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        ctx.set_timing(True)
        ctx.reset_stats()
        for _ in range(5):
            batch.run_bytes(ctx, shape)
        ctx.set_timing(False)
        ks = {k: round(ctx.kernel_stats(k)[1] / 5, 4) for k in KERNELS}
        print(json.dumps({"B": B, "logn": logn, "ladder": os.environ.get("LADDER", "auto"), "twist": os.environ.get("TWIST", "auto"),
                          "split": os.environ.get("SPLIT", "auto"), "ms_per_batch": round(ms, 4), "proofs_per_s": round(B / ms * 1e3, 1),
                          "kernels_ms": ks, "status_nonzero": int((batch.status != 0).sum().item())}), flush=True)
        del batch
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
