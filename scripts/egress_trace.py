import sys; sys.path.insert(0, ".")
import numpy as np
from tests import util
lens = util.zipf_lengths(); payload = util.splitmix64(0x5EED, int(lens.sum()))
util.egress_stacks(payload[:4096], [64]*64, 1 << 20, 10240)
for T in [int(a) for a in sys.argv[1:]]:
    t = np.zeros(2); util.egress_stacks(payload, lens, 1 << 20, 10240, times=t, raw=True, threads=T)
    print("T", T, t, "GiB/s", lens.sum() / t.sum() / 2**30, file=sys.stderr, flush=True)
