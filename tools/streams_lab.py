"""Lab: bench.py's steps (n=10, m=3, 1M trials, staged inputs) one at a time vs
alternating over 2 or 3 ctxs, each on its own ctx stream (ba_ctx_stream).

    python tools/streams_lab.py [K]        # K steps per timed pass (default 20)
    MODE=events|setstream|both ...        # bench.py's event/stream plumbing variants

Prints trials/s per number of steps in flight, three passes each; every pass's
counters must equal K x 1M trials.  Round 2 on one MI355X: 1.99e10 (1), 2.43e10
(2), 2.42e10 (3) at K=20; 2.00e10 / 2.53e10 / 2.51e10 at K=60."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # repo root
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))
import torch
from ba_amd import lib as L
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
n, m, B, K = 10, 3, 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 20
NS = 4
engs = [L.Engine(0) for _ in range(NS)]
sts = [torch.cuda.ExternalStream(e.stream(), device=dev) for e in engs]
nslot = K + 8
fb = torch.empty((nslot, B), dtype=torch.int32, device=dev)
ob = torch.empty((nslot, B), dtype=torch.uint8, device=dev)
gp = [L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM, L.ATTACK, L.ENGINE_AUTO, i * B) for i in range(nslot)]
sp = [L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 3, L.ORDER_GIVEN, L.ATTACK, L.ENGINE_AUTO, i * B) for i in range(nslot)]
for i in range(nslot):
    engs[0].gen_inputs_device(gp[i], B, d_faulty=fb[i].data_ptr(), d_order=ob[i].data_ptr(), stream=sts[0].cuda_stream)
torch.cuda.synchronize()
dec = [torch.empty(B, dtype=torch.int64, device=dev) for _ in range(NS)]
out = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(NS)]
cnt = torch.zeros(16, dtype=torch.int64, device=dev)
MODE = os.environ.get("MODE", "plain")
if MODE in ("setstream", "both"):
    torch.cuda.set_stream(sts[0])
def run(ns, base):
    cnt.zero_(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    if MODE in ("events", "both"):
        ev0 = torch.cuda.Event(enable_timing=True); ev0.record(sts[0])
        for j in range(1, ns): sts[j].wait_event(ev0)
    for i in range(K):
        j = i % ns
        engs[j].run_device(sp[base + i], B, d_faulty=fb[base + i].data_ptr(), d_order=ob[base + i].data_ptr(),
                           d_decisions=dec[j].data_ptr(), d_outcome=out[j].data_ptr(), d_counters=cnt.data_ptr(),
                           stream=sts[j].cuda_stream)
    if MODE in ("events", "both"):
        for j in range(1, ns): sts[0].wait_stream(sts[j])
    torch.cuda.synchronize()
    return time.perf_counter() - t0, int(cnt[0].item())
t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    for ns in (1, 2, 3):
        run(ns, 0)
res = {}
for rep in range(3):
    for ns in (1, 2, 3):
        dt, tr = run(ns, 0)
        assert tr == K * B, tr
        res.setdefault(ns, []).append(K * B / dt)
print(json.dumps({"mode": MODE, "K": K, "trials_per_s": {k: [round(x / 1e10, 4) for x in v] for k, v in res.items()}}))
