"""Diagnostic: config-5 stream through the local transport, per step, with and without
combining, sync and pipelined; prints the first mismatches (GPU)."""
import sys
import numpy as np
sys.path[:0] = ["api-ratelimit_amd", "tests", "oracle"]
import torch  # noqa
import hiprl, oracle, workload, streams  # noqa
from test_gpu_combining import engines, Bufs, check, run_steps  # noqa


def run(G, combine, mode, steps_n=6, per=1500):
    es = engines(G, per * G, rules=workload.CONFIG5_RULES)
    r = hiprl.Router(es, max_desc=per, combine=combine)
    o = oracle.Oracle()
    o.load_rules(workload.CONFIG5_RULES)
    steps = [[workload.config5_batch(s * G + g, per, 3000, batches_per_s=2, seed=5 + g) for g in range(G)]
             for s in range(steps_n)]
    steps = [[hiprl.Batch(b.blob, b.off, b.rule, b.req_of, np.full(b.n_req, 1_700_000_000 - 37 + s // 2, np.int64),
                          b.hits) for b in row] for s, row in enumerate(steps)]
    try:
        run_steps(r, steps, o, mode, f"G={G} combine={combine} {mode}")
        print("OK", G, combine, mode, r.stats()["combined_steps"], flush=True)
    except AssertionError as ex:
        print("FAIL", G, combine, mode, str(ex)[:300], r.stats(), flush=True)
    r.close()


for G in (2, 8):
    for combine in (False, True):
        for mode in ("sync", "pipelined"):
            run(G, combine, mode)
