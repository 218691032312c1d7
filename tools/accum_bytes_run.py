"""Driver for profiling the accumulator leg of bench.py: B simple-example
proofs (BN254, k = 17 by default) from their serialized bytes through
pm_accum_batch_proofs_device, REPS times (rocprofv3 --pmc / --kernel-trace
wraps it: tools/gpu_pmc_acc.sh).  Env: B, LOGN, REPS, DECODED=1 (the
decoded-input entry pm_accum_batch_transcript_device instead)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd")]
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402
import workloads as Wk  # noqa: E402


def main():
    B, logn, reps = int(os.environ.get("B", "256")), int(os.environ.get("LOGN", "17")), int(os.environ.get("REPS", "20"))
    ctx = H.Context(0)
    shape = Wk.simple_example_shape(ctx, H.BN254, logn)
    batch = Wk.SyntheticBatch(ctx, shape, B)
    batch.to_proof_bytes(shape)
    decoded = os.environ.get("DECODED") == "1"
    for _ in range(reps):
        if decoded:
            batch.run(ctx, shape)
        else:
            batch.run_bytes(ctx, shape)
    torch.cuda.synchronize()
    print("status_nonzero", int((batch.status != 0).sum().item()), flush=True)


if __name__ == "__main__":
    main()
