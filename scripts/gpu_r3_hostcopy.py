"""Host memcpy capability of the box: N threads copying 1 MiB pieces into pageable and pinned memory."""
import ctypes as C
import threading
import time
import numpy as np
import torch

src = np.random.randint(0, 255, 8 << 20, dtype=np.uint8)
for kind in ("pageable", "pinned"):
    for th in (1, 2, 4, 8):
        per = (1 << 30) // th
        dsts = []
        for t in range(th):
            if kind == "pinned":
                d = torch.empty(per, dtype=torch.uint8).pin_memory()
                d.zero_()
                dsts.append((d, d.data_ptr()))
            else:
                d = np.zeros(per, dtype=np.uint8)
                dsts.append((d, d.ctypes.data))

        def run(t):
            base = dsts[t][1]
            for rep in range(2):
                for i in range(per >> 20):
                    C.memmove(base + (i << 20), src.ctypes.data + ((i % 8) << 20), 1 << 20)

        ths = [threading.Thread(target=run, args=(t,)) for t in range(th)]
        t0 = time.perf_counter()
        [x.start() for x in ths]
        [x.join() for x in ths]
        el = time.perf_counter() - t0
        print(f"{kind} threads={th}: {2 * (1 << 30) / el / 1e9:.1f} GB/s", flush=True)
        del dsts
