"""Ad-hoc GPU parity probe: config-2 batches of several sizes, bucketed vs LSD vs oracle."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "api-ratelimit_amd"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402

import hiprl  # noqa: E402
import oracle  # noqa: E402
import workload  # noqa: E402

for d, N in [(int(a.split(":")[0]), int(a.split(":")[1])) for a in sys.argv[1:]]:
    b = workload.config2_batch(0, d=d, N=N)
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=True)
    o.load_rules(workload.CONFIG2_RULES)
    ost, othr = o.submit(b, threads=8)
    for lsd in (False, True):
        e = hiprl.Engine(log2_slots=(23, 12, 12, 12), max_batch_desc=d, max_batch_req=d,
                         max_blob_bytes=int(b.blob.shape[0]) + 64, lsd_only=lsd)
        e.load_rules(workload.CONFIG2_RULES)
        gst, gthr = e.submit(b)
        bad = np.nonzero(ost != gst)[0]
        print(f"d={d} N={N} lsd={lsd} stats={e.stats()} bad={len(bad)} thr_bad={(othr != gthr).sum()}", flush=True)
        for i in bad[:3]:
            k = bytes(b.blob[b.off[i]:b.off[i + 1]])
            rank_keys = np.array([bytes(b.blob[b.off[j]:b.off[j + 1]]) for j in range(d)], dtype=object) \
                if "rank_keys" not in dir() else rank_keys
            same = list(np.nonzero(rank_keys == k)[0])
            print("  idx", i, k, "oracle", ost[i], "gpu", gst[i], "same-key idx", same[:12], flush=True)
            for j in same[:12]:
                print("     ", j, ost[j], gst[j])
        del e
