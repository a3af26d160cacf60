"""Debug helper: do the loads' "negative" offsets read the previous channel?
Channel 0 is 1000.0 everywhere, channel 1 random; outputs of channel 1 next
to its start against the oracle, for both methods."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import conftest  # noqa: F401  (paths)
import lcfir as lc
import oracle as om
om.load()
from test_gpu_parity import gpu_filter_channels

for method, ntaps, n in [("direct", 801, 20000), ("direct", 15, 20000), ("direct", 4001, 50000),
                         ("fft", 4003, 50000), ("fft", 4001, 50000)]:
    rng = np.random.default_rng(ntaps)
    x = (rng.integers(-2**23, 2**23, size=(2, n)) / 2.0**23).astype(np.float32)
    x[0] = 1000.0
    taps = om.design_lowcut(20.0, 48000.0, ntaps)
    flt = lc.Filter(taps, method=method)
    y, pk = gpu_filter_channels(lc, flt, x)
    ref = om.filter_channel(x[1], taps, om.MODE_FMA)
    d = np.abs(y[1].astype(np.float64) - ref)
    bad = np.nonzero(d > 1e-5)[0]
    print(method, ntaps, "bad", bad.size, "range", (bad.min(), bad.max()) if bad.size else None,
          "maxdiff", d.max(), "y0", y[1][:3].tolist(), "ref0", ref[:3].tolist(), flush=True)
