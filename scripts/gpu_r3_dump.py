"""Dump the throughput engine's frames for a few inputs next to the model's (debug aid)."""
import os, sys, random, pickle
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import librdkafka_amd as L
from test_gpu_lz4 import _fast_compress, _fast_inputs
import units_model
L.init(0)
inputs = _fast_inputs(45, 20)
frames = _fast_compress(L, inputs)
bad = []
for i, (b, fr) in enumerate(zip(inputs, frames)):
    if fr != units_model.frame(b):
        bad.append(i)
print("mismatching inputs:", bad, [len(inputs[i]) for i in bad])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "dump_frames.pkl"), "wb") as f:
    pickle.dump({i: frames[i] for i in bad[:4]}, f)
