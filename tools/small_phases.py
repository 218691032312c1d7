"""Host phases of the small-MSM path (round 6): the drop-in
pm_msm_ctx with host scalars and FRESH host bases (the verifier's MSMs over
proof points) at n = 1, 32, 4096, timed per call from Python and, inside the
library, per phase (pm_ctx_set_timing_filter "small_host": no kernel is
event-timed, so the call runs exactly as untimed): small_stage (copy into the
pinned staging buffer), small_launch (buffers, counters, launches queued),
small_wait (launch -> completion flag), host_tail (33-window Horner),
small_finish (affine conversion).  The rest of a call is ctypes / numpy /
digest / bookkeeping.  Usage: python tools/small_phases.py > out.jsonl"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import halo2_amd as H  # noqa: E402
import msm_ref  # noqa: E402

PH = ("small_stage", "small_launch", "small_wait", "host_tail", "small_finish")


def main():
    curve = H.PALLAS
    ctx = H.Context(0)
    S = msm_ref.synth_scalars(curve, 0x5EED, 0, 1 << 14, threads=8)
    B = msm_ref.synth_bases(curve, 0xA11CE, 0, 1 << 14, threads=8)
    for n in [int(x) for x in os.environ.get("NS", "1,32,4096").split(",")]:
        reps = 40
        s = np.ascontiguousarray(S[:n])
        fresh = [np.ascontiguousarray(B[k + 1:k + 1 + n]) for k in range(reps)]
        # settle: ~20 ms of untimed calls (after the host-side input synthesis
        # the GPU idles and its clocks drop; the first loop ran 248 us per call
        # at n = 1 against 57 us warm)
        warm = [np.ascontiguousarray(B[len(B) - n - 1 - k:len(B) - 1 - k]) for k in range(2)]  # own sets
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.02:
            for bf in warm:
                ctx.msm(curve, s, bf)
        t0 = time.perf_counter()
        for bf in fresh:
            ctx.msm(curve, s, bf)
        py_us = (time.perf_counter() - t0) * 1e6 / reps
        ctx.set_timing(True, only="small_host")
        ctx.reset_stats()
        t0 = time.perf_counter()
        for bf in fresh:
            ctx.msm(curve, s, bf)
        timed_us = (time.perf_counter() - t0) * 1e6 / reps
        ph = {k: round(ctx.kernel_stats(k)[1] * 1e3 / reps, 2) for k in PH}
        ctx.set_timing(False)
        # the bare ctypes + numpy cost of one call, measured on pm_point_add
        a = np.zeros(8, np.uint64)
        t0 = time.perf_counter()
        for _ in range(200):
            H.point_add(curve, a, a)
        ffi_us = (time.perf_counter() - t0) * 1e6 / 200
        print(json.dumps({"n": n, "py_us_per_call": round(py_us, 1), "timed_us_per_call": round(timed_us, 1),
                          "phases_us": ph, "rest_us": round(timed_us - sum(ph.values()), 1),
                          "ctypes_call_us": round(ffi_us, 2)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
