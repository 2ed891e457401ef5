"""stream_handle() against torch.cuda.current_stream() (tools only; round 6): same handle, per-call cost."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from adaptive_amd import _lib  # noqa: E402
assert _lib.stream_handle() == torch.cuda.current_stream().cuda_stream
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    assert _lib.stream_handle() == s.cuda_stream, (_lib.stream_handle(), s.cuda_stream)
t0 = time.perf_counter()
for _ in range(10000): _lib.stream_handle()
t1 = time.perf_counter()
for _ in range(10000): torch.cuda.current_stream().cuda_stream
t2 = time.perf_counter()
print(f"stream_handle {(t1-t0)/1e4*1e6:.2f} us, current_stream {(t2-t1)/1e4*1e6:.2f} us")
