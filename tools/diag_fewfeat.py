import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from cocoa_amd import Engine
from oracle import oracle
from tests.test_gpu_multidevice import _tiny, odata
tr = _tiny(3)
od = odata(tr)
run = oracle.Run(od, "cocoa+", tr.n, 10, 1e-2)
ws = []
for t in range(1, 6):
    run.round(t)
wr = run.w()
for rep in range(3):
    for devs in ([0] * 4, None):
        e = Engine(devices=devs, strict=False) if devs else Engine(strict=False)
        e.set_train(tr)
        e.set_test(tr)
        e.init("cocoa+", tr.n, 5, 10, 1e-2)
        for t in range(1, 6):
            e.round(t)
        print(rep, "members" if devs else "single", e.plan()["solver"], e.plan().get("gram_mirror"), np.max(np.abs(e.w() - wr)), flush=True)
