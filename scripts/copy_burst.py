# The streaming-copy yardstick (gh_bw_copy) in bursts of 3, 20, 100 and 400 launches after
# idle, to tell the decode's first-launches dip (clock settling under load) from a property
# of the decode kernel.  Run under rocprofv3 --kernel-trace; summarise with trace_series.py.
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cse375-finalproj-huffman-decoding_amd"))
import torch
import gaphuff as gh
nbytes = 2_012_499_128  # the cfg4 decode's algorithmic bytes (read + write)
half = nbytes // 2 // 16 * 16
src = torch.empty(half, dtype=torch.uint8, device="cuda")
dst = torch.empty(half, dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
for reps in (3, 20, 100, 400, 3):
    time.sleep(0.5)
    ms = gh.bw_copy(dst.data_ptr(), src.data_ptr(), half, stream, reps=reps)
    print(f"copy reps={reps:4d} ms={ms:.4f} GB/s={2 * half / ms / 1e6:.0f}", flush=True)
