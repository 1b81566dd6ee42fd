import time, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
t0 = time.time()
def log(*a):
    print(f"[{time.time()-t0:7.2f}s]", *a, flush=True)
from charon_amd import engine as eng
log("import")
e = eng.Engine(0)
log("engine")
from tools.workload import make_batch
b = make_batch(e, 16, 3, 4, seed=1)
log("make_batch (sign kernels)")
r = e.run(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
          duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
log("run", (r.partial_status == 1).all(), (r.duty_status == 0).all())
log("timings", e.timings())
