import sys, os
sys.path.insert(0, os.getcwd())
import torch
os.environ.setdefault("P2PFL_CHECK_FINITE", os.environ.get("CF", "0"))
from tests.test_gpu_fused_cnn import test_fused_and_torch_peers_federate
ok = 0
for i in range(6):
    try:
        test_fused_and_torch_peers_federate()
        ok += 1
        print(f"iter {i}: ok", flush=True)
    except AssertionError as e:
        print(f"iter {i}: FAIL {e}", flush=True)
        from p2pfl_amd.utils import finite
        print("first failure:", finite.FIRST_FAILURE[:3], flush=True)
        break
print("ok", ok)
