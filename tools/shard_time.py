"""One shard-batch point of bench.py's sweep (S bytes per shard, ~256 MB of shards): encode_shards +
decode_shards per-call times.  Usage: shard_time.py S [steps]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ezpwd-reed-solomon_amd"))
import torch
import bench
import ezrs

S = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
codec = ezrs.Codec.rs(255, 223)
gen = torch.Generator(device="cuda").manual_seed(1)
print(bench.shard_point(codec, S, steps, 10, gen))
