"""Feed the edge-line corpus one line at a time (GPU), printing each line first."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_parity import EDGE_CFG, edge_lines, S  # noqa: E402
from tests.parity import Pair  # noqa: E402

t = 1700000000
pair = Pair(EDGE_CFG)
data = edge_lines(t)
for i, ln in enumerate(data.split(b"\n")[:-1]):
    print(i, repr(ln), flush=True)
    pair.feed(ln + b"\n", t * S)
print("whole", flush=True)
pair.feed(data, t * S)
print("ok", flush=True)
