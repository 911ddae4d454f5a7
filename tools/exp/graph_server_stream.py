"""Experiment: capture the N>1 (size-1 xGMI arena) sparse-LR step as hipGraphs
with the server stream kept in the capture.  argv[1]: prio (the engine's
top-priority server stream), normal (a default-priority stream instead),
none (retired: the default)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
os.environ["SS_PULL_AHEAD"] = "0"
os.environ["SS_XGMI_TIMEOUT"] = "20"
mode = sys.argv[1]
import torch  # noqa: E402

from test_gpu_models import _graph_worker  # noqa: E402
from swiftsnails_amd.parallel.xgmi import XgmiTransport  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
a, ta = _graph_worker("lr", dev, transport=XgmiTransport(0, 1, dev, None))
if mode == "normal":
    torch.cuda.synchronize()
    a.engine.server_stream = torch.cuda.Stream(device=dev)
# (models/base.py enable_graph retires the server stream before a capture;
# this experiment patched that out to capture it, forked and joined: both
# priorities crashed inside hipStreamEndCapture, round 6)
for _ in range(2):
    a.step()
print("eager ok", a.mean_loss(), flush=True)
assert a.enable_graph()
print("captured", flush=True)
for _ in range(3 * a._gper):
    a.step()
torch.cuda.synchronize()
a.engine.check()
print("replayed", mode, a.mean_loss(), flush=True)
