"""Launch k_om3w<10> (staged inputs, bench.py's workload: n=10, m=3, 1,048,576
trials, seed 0xBA5EED) `--reps` times on one stream, with no result checks: the
PMC driver for lab ablation builds whose results are wrong by design
(tools/gpu_session.sh `bank`; BA_HIP_LIB names the build)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))

import torch  # noqa: E402

from ba_amd import lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=4)
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng = L.Engine(0)
s = eng.stream()
T = 1 << 20
pr = L.make_params(10, 3, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM, L.ATTACK, L.ENGINE_AUTO, 0)
pg = L.make_params(10, 3, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 3, L.ORDER_GIVEN, L.ATTACK, L.ENGINE_AUTO, 0)
fb = torch.empty(T, dtype=torch.int32, device=dev)
ob = torch.empty(T, dtype=torch.uint8, device=dev)
dec = torch.empty(T, dtype=torch.int64, device=dev)
oc = torch.empty(T, dtype=torch.uint8, device=dev)
cnt = torch.zeros(16, dtype=torch.int64, device=dev)
eng.gen_inputs_device(pr, T, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), stream=s)
for _ in range(a.reps):
    eng.run_device(pg, T, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), d_decisions=dec.data_ptr(),
                   d_outcome=oc.data_ptr(), d_counters=cnt.data_ptr(), stream=s)
torch.cuda.synchronize()
print("launches", a.reps, "trials", int(cnt[0].item()))
eng.close()
