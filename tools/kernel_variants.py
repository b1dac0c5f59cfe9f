"""Time library variants (tools/variants/lib_*.so) on config-3 batches; per-kernel µs per batch.
Also checks every variant's outputs equal the first variant's (bit-exact)."""
import glob
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))
import hiprl  # noqa: E402
import workload  # noqa: E402

libs = sorted(glob.glob(str(ROOT / "tools" / "variants" / "lib_*.so")))
if len(sys.argv) > 1:
    libs = [l for l in libs if any(Path(l).stem.endswith(x) for x in sys.argv[1:])]
nb = 8
hbs = [workload.config3_batch(b) for b in range(nb)]
dev = torch.device("cuda", 0)
dbs = []
for hb in hbs:
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dbs.append([t(hb.blob), t(hb.off.view(np.int32)), t(hb.rule.view(np.int32)), t(hb.req_of.view(np.int32)),
                t(hb.now), t(hb.hits.view(np.int32))])
torch.cuda.synchronize()
ref = None
for lp in libs:
    eng = hiprl.Engine(log2_slots=(22, 24, 25, 12), max_batch_desc=10**6, max_blob_bytes=40 * 10**6, lib_path=lp)
    eng.load_rules(workload.CONFIG3_RULES)
    out = torch.empty(10**6 * 20, dtype=torch.uint8, device=dev)
    thr = torch.empty(10**6, dtype=torch.int32, device=dev)
    outs = []
    for i, (hb, db) in enumerate(zip(hbs, dbs)):
        if i == 2:
            eng.set_timing(True)
        eng.submit_device_async(hb.n_desc, hb.n_req, int(hb.off[-1]), [x.data_ptr() for x in db], out.data_ptr(),
                                thr.data_ptr())
        eng.wait()
        outs.append(out.cpu().numpy().copy())
    kt = eng.kernel_times()
    tot = sum(v[0] for v in kt.values()) / (nb - 2) * 1e3
    desc = " ".join(f"{k}={v[0] / (nb - 2) * 1e3:.1f}" for k, v in kt.items() if v[1])
    same = "ref" if ref is None else ("same" if all(np.array_equal(a, b) for a, b in zip(ref, outs)) else "DIFF")
    if ref is None:
        ref = outs
    print(f"{Path(lp).stem}: total {tot:.1f} us/batch [{same}]  {desc}", flush=True)
    eng.close()
