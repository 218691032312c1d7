"""Host planning time of the accumulator call (round 6): pm_accum_batch_proofs_device
on B simple-example proofs (BN254, k = 17), timing filter "accum_host" (no
kernel events): accum_plan_host = entry of the accumulator's plan -> the
ladder's launch, and the wall time per call.  Usage: python tools/accum_host_phases.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd")]
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402
import workloads as Wk  # noqa: E402


def main():
    ctx = H.Context(0)
    shape = Wk.simple_example_shape(ctx, H.BN254, 17)
    for B in [int(x) for x in os.environ.get("BS", "16,256,1024").split(",")]:
        batch = Wk.SyntheticBatch(ctx, shape, B)
        batch.to_proof_bytes(shape)
        for _ in range(5):
            batch.run_bytes(ctx, shape)
        torch.cuda.synchronize()
        ctx.set_timing(True, only="accum_host")
        ctx.reset_stats()
        t0 = time.perf_counter()
        for _ in range(20):
            batch.run_bytes(ctx, shape)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / 20
        n, tot = ctx.kernel_stats("accum_plan_host")
        ctx.set_timing(False)
        print(json.dumps({"B": B, "ms_per_batch": round(ms, 4), "plan_host_us": round(tot * 1e3 / max(1, n), 2)}),
              flush=True)


if __name__ == "__main__":
    main()
