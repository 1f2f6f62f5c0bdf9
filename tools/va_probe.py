#!/usr/bin/env python3
"""How much device virtual address space can one process reserve? (qk_out_alloc's ceiling.)

qk_out_alloc never hands a freed mapping's address range out again (its translations outlived the
mapping), so a long-lived process retires one range per freed output. This probe
reserves ranges with exactly qk_out_alloc's call (hipMemAddressReserve(size, align = 1 GiB, addr 0,
flags 0)) until the runtime refuses or a cap is reached, then frees them all. No physical memory is
created and nothing is mapped or launched.

    python tools/va_probe.py [--size-gib 32] [--cap-tib 1024] > profiles/r06_va_probe.json
"""
import argparse
import ctypes
import json
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-gib", type=int, nargs="+", default=[32, 4, 512])
    ap.add_argument("--cap-tib", type=float, default=1024.0, help="stop after this much reserved (TiB)")
    args = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemAddressReserve.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_ulonglong]
    hip.hipMemAddressFree.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    hip.hipSetDevice.argtypes = [ctypes.c_int]
    hip.hipGetErrorString.restype = ctypes.c_char_p
    assert hip.hipSetDevice(0) == 0
    out = {"probe": "hipMemAddressReserve(size, 1 GiB, NULL, 0) until failure or cap", "runs": []}
    for gib in args.size_gib:
        size = gib << 30
        held = []
        err = None
        t0 = time.perf_counter()
        cap = int(args.cap_tib * (1 << 40))
        while len(held) * size < cap:
            p = ctypes.c_void_p()
            e = hip.hipMemAddressReserve(ctypes.byref(p), size, 1 << 30, None, 0)
            if e != 0:
                err = f"{e}: {hip.hipGetErrorString(e).decode()}"
                break
            held.append(p.value)
        dt = time.perf_counter() - t0
        lo = min(held) if held else 0
        hi = max(held) + size if held else 0
        for p in held:
            hip.hipMemAddressFree(ctypes.c_void_p(p), size)
        out["runs"].append({"size_gib": gib, "reservations": len(held), "reserved_tib": len(held) * size / 2**40,
                            "stopped_by": err or f"cap {args.cap_tib} TiB", "seconds": round(dt, 3),
                            "lowest": hex(lo), "highest_end": hex(hi)})
        print(json.dumps(out["runs"][-1]), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
