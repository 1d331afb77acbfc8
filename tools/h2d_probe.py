#!/usr/bin/env python3
"""Does an H2D copy from pinned host memory return before it completes?  Host time of the
enqueue vs the copy's device time, for torch's copy_(non_blocking=True) and for
hipMemcpyAsync called directly, 478 MB (one bench input block) and 32 MB."""
import ctypes as C
import time

import torch


def main():
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    s = torch.cuda.Stream()
    for nb in (32 << 20, 478281400):
        h = torch.empty(nb, dtype=torch.uint8).pin_memory()
        d = torch.empty(nb, dtype=torch.uint8, device="cuda")
        print("pinned", h.is_pinned(), flush=True)
        for way in ("torch", "hip"):
            for rep in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if way == "torch":
                    with torch.cuda.stream(s):
                        d.copy_(h, non_blocking=True)
                else:
                    rc = hip.hipMemcpyAsync(C.c_void_p(d.data_ptr()), C.c_void_p(h.data_ptr()), nb, 1,
                                            C.c_void_p(s.cuda_stream))
                    assert rc == 0
                t1 = time.perf_counter()
                s.synchronize()
                t2 = time.perf_counter()
                print("%s %d MB: enqueue %.3f ms, done %.3f ms" % (way, nb >> 20, (t1 - t0) * 1e3,
                                                                  (t2 - t0) * 1e3), flush=True)


if __name__ == "__main__":
    main()
