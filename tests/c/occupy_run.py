"""TEST SUPPORT ONLY: hold `blocks` CUs' worth of the GPU for `seconds` from a process of its own (tests/c/occupy.hip).
Prints RUNNING once every holding workgroup runs, DONE when the kernel has ended.
    python tests/c/occupy_run.py <blocks> <seconds>   (blocks 0: half the CUs)"""
import ctypes as ct
import os
import sys
import time


def main():
    occ = ct.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libocc.so"))
    blocks, secs = int(sys.argv[1]), float(sys.argv[2])
    if blocks <= 0:
        blocks = max(1, occ.occ_cus() // 2)
    host, dev = ct.POINTER(ct.c_int)(), ct.POINTER(ct.c_int)()
    assert occ.occ_alloc(blocks, ct.byref(host), ct.byref(dev)) == 0
    assert occ.occ_launch(None, blocks, ct.c_double(secs), host, dev) == 0
    t0 = time.time()
    while sum(host[i] for i in range(blocks)) < blocks:
        if time.time() - t0 > 30:
            print("NOSTART", flush=True)
            return 1
        time.sleep(0.0005)
    print("RUNNING", blocks, flush=True)
    rc = occ.occ_sync()
    occ.occ_free(host)
    print("DONE", rc, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
