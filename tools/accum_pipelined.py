"""Two accumulator batches in flight (diagnostic): B = 256 proofs from bytes
(pm_accum_batch_proofs_device, the bench's accumulator leg) on one context,
then on two contexts (each its own HIP streams and workspace) driven by two
host threads.  The batch's kernels are latency-bound chains that leave most
SIMDs idle, so a second batch in flight measures how much of
the chip one batch leaves unused.  Prints one JSON line per mode."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo2-aggregation_amd"))
import torch  # noqa: E402

import halo2_amd as H  # noqa: E402
import workloads as Wk  # noqa: E402


def main():
    B = int(os.environ.get("B", "256"))
    logn = int(os.environ.get("LOGN", "17"))
    steps = int(os.environ.get("STEPS", "40"))
    ctxs = [H.Context(0), H.Context(0)]
    shape = Wk.simple_example_shape(ctxs[0], H.BN254, logn)
    batches = [Wk.SyntheticBatch(ctxs[0], shape, B, i0=i * B) for i in range(2)]
    for b in batches:
        b.to_proof_bytes(shape)
    for c, b in zip(ctxs, batches):
        for _ in range(5):
            b.run_bytes(c, shape)
    torch.cuda.synchronize()
    ref = [b.quads.clone() for b in batches]

    t0 = time.perf_counter()
    for _ in range(steps):
        batches[0].run_bytes(ctxs[0], shape)
    torch.cuda.synchronize()
    one = (time.perf_counter() - t0) / steps
    print(json.dumps({"mode": "one_context", "B": B, "ms_per_batch": round(one * 1e3, 4),
                      "proofs_per_s": round(B / one, 1)}), flush=True)

    errs = []

    def loop(i):
        try:
            for _ in range(steps):
                batches[i].run_bytes(ctxs[i], shape)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=loop, args=(i,)) for i in range(2)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    two = time.perf_counter() - t0
    same = all(torch.equal(r, b.quads) for r, b in zip(ref, batches))
    ok = all(int((b.status != 0).sum().item()) == 0 for b in batches)
    print(json.dumps({"mode": "two_contexts_two_threads", "B": B, "batches": 2 * steps,
                      "ms_per_batch": round(two * 1e3 / (2 * steps), 4),
                      "proofs_per_s": round(2 * steps * B / two, 1), "quads_match": same, "status_ok": ok,
                      "errors": errs}), flush=True)


if __name__ == "__main__":
    main()
