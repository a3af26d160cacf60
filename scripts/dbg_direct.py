"""Debug helper: direct method vs the strict-fma oracle on small channels,
printing where outputs differ (tile = 4096 outputs)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "audio-fir-filter_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import lcfir as lc
import oracle as om
om.load()
from test_gpu_parity import gpu_filter_channels

for ntaps, n in [(15, 20000), (801, 20000), (4001, 50000), (19201, 100000)]:
    rng = np.random.default_rng(ntaps)
    x = (rng.integers(-2**23, 2**23, size=(2, n)) / 2.0**23).astype(np.float32)
    taps = om.design_lowcut(20.0, 48000.0, ntaps)
    flt = lc.Filter(taps, method="direct")
    y, pk = gpu_filter_channels(lc, flt, x)
    for c in range(2):
        ref = om.filter_channel(x[c], taps, om.MODE_FMA)
        bad = np.nonzero(y[c] != ref)[0]
        tiles = np.unique(bad // 4096)
        print(ntaps, n, c, "bad", bad.size, "first", bad[:5].tolist(), "tiles", tiles[:20].tolist(),
              "lanes", np.unique((bad % 4096) // 16)[:20].tolist(), "y", y[c][bad[:3]].tolist(), "ref", ref[bad[:3]].tolist(),
              flush=True)
