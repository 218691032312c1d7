"""Per-kernel timing of the batch accumulator (diagnostic): synthetic proofs
generated on the device (points [a]G, scalars / challenges uniform)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import accum_util as U  # noqa: E402
import halo2_amd as H  # noqa: E402

KERNELS = ["transcript", "acc_ladder", "acc_scalars", "acc_termmul", "acc_sum"]


def main():
    curve = int(os.environ.get("CURVE", "2"))
    ctx = H.Context(0)
    splits = [int(x) for x in os.environ.get("SPLITS", "-1").split(",")]
    extra = [("simple", 17, int(b)) for b in os.environ.get("BATCHES", "").split(",") if b]
    for split, shape, log_n, B in [(sp,) + c for sp in splits for c in [("simple", 14, 16), ("simple", 17, 256), ("simple", 17, 4096), ("rich", 17, 256)] + extra
                                          if os.environ.get("CASES", "all") == "all" or "%s:%d" % (c[0], c[2]) in
                                          os.environ["CASES"].split(",")]:
        ctx.set_accum_split(split)
        C, sh, _ = U.make_case(curve, shape, log_n, 0, 0x5EED)
        ps = U.to_product_shape(curve, sh)
        npts, nsc, _ = ps.layout()
        dev = torch.device("cuda", 0)
        pts = torch.empty((B, npts, 8), dtype=torch.int64, device=dev)
        scs = torch.empty((B, nsc, 4), dtype=torch.int64, device=dev)
        chs = torch.empty((B, 7, 4), dtype=torch.int64, device=dev)
        ctx.synth_bases(curve, 0xA11CE, 0, B * npts, pts.data_ptr())
        ctx.synth_scalars(curve, 0x5CA1A, 0, B * nsc, scs.data_ptr())
        ctx.synth_scalars(curve, 0xC4A1, 0, B * 7, chs.data_ptr())
        dq = torch.empty((B, 4, 8), dtype=torch.int64, device=dev)
        dh = torch.empty((B, 4), dtype=torch.int64, device=dev)

        fused = os.environ.get("TRANSCRIPT", "1") == "1"
        vk = U.np.array([1, 2, 3, 4], dtype=U.np.uint64)

        def run():
            if fused:   # challenges replayed from the Blake2b transcript on the device
                ctx.accum_batch_transcript_device(ps, B, vk, pts.data_ptr(), scs.data_ptr(), chs.data_ptr(),
                                                  dq.data_ptr(), dh.data_ptr())
            else:
                ctx.accum_batch_device(ps, B, pts.data_ptr(), scs.data_ptr(), chs.data_ptr(), dq.data_ptr(),
                                       dh.data_ptr())

        run()
        reps = int(os.environ.get("REPS", "20"))
        ts = []
        for _ in range(reps):
            t = time.time()
            run()
            ts.append(time.time() - t)
        wall = sorted(ts)[len(ts) // 2]  # median of single calls
        ctx.set_timing(True)
        ctx.reset_stats()
        for _ in range(reps):
            run()
        ctx.set_timing(False)
        ks = {k: round(ctx.kernel_stats(k)[1] / reps, 4) for k in KERNELS}
        print(json.dumps({"split": split, "transcript": fused, "shape": shape, "log_n": log_n, "B": B, "wall_ms": round(wall * 1e3, 3),
                          "proofs_per_s": round(B / wall, 1), "kernels_ms": ks}), flush=True)


if __name__ == "__main__":
    main()
