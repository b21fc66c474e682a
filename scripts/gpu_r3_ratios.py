import random, sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))); sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))), "tests"))
import librdkafka_amd as L, oracle
from librdkafka_amd import workload as W
import importlib.util
spec = importlib.util.spec_from_file_location("t", __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))), "tests", "test_gpu_lz4.py"))
t = importlib.util.module_from_spec(spec); spec.loader.exec_module(t)
L.init(0)
rnd = random.Random(43)
words = [bytes(rnd.choice(b"abcdefghij") for _ in range(rnd.randrange(2, 10))) for _ in range(500)]
text = b" ".join(rnd.choice(words) for _ in range(300000))[:1 << 20]
names = ["json 1MiB", "json 64K", "json 1MiB b", "word soup", "rep3000"]
inputs = [W.gen_json(1 << 20, 42), W.gen_json(65536, 7), W.gen_json(1 << 20, 5), text, (rnd.randbytes(3000) * 400)[:1 << 20]]
from librdkafka_amd import workload
msgs = None
pt = bytes(W.PERF_PATTERN) if hasattr(W, "PERF_PATTERN") else None
if pt: names.append("perf pattern x"); inputs.append((pt * 20000)[:1 << 20])
frames = t._fast_compress(L, inputs, False)
for nm, b, fr in zip(names, inputs, frames):
    ref = oracle.rdk_lz4_compress(b)[1]
    print(f"{nm:14s} gpu {len(b)/len(fr):7.3f} ref {len(b)/len(ref):7.3f} rel {len(ref)/len(fr):.4f}", flush=True)
