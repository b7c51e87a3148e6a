import time, json, sys
sys.path.insert(0, '.')
from firedancer_amd import ed25519
t0 = time.perf_counter(); e = ed25519.Engine(0, max_chunk=1 << 20); t1 = time.perf_counter()
e2 = ed25519.Engine(0, max_chunk=1 << 12); t2 = time.perf_counter()
print(json.dumps({"first_engine_s": t1 - t0, "second_engine_s": t2 - t1}))
