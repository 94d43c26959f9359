"""Probe (no faults): does a registration of CALLER host memory outlive the call that made it?

For each way host memory reaches the GPU -- torch's own pageable copies, the library's host APIs
(rh_segments_read_host / rh_crc32c_verify_host: caller arrays handed to the runtime), an explicit
rh_host_register / rh_host_unregister pair -- this prints whether the HIP runtime still knows the
caller's address range after the call returned (hipPointerGetAttributes / hipMemPtrGetInfo).  A
range the runtime still holds pinned while the caller frees the memory is a userptr mapping whose
pages go away under it."""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from ratis_amd import _lib, engine  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch already loaded (same SONAME)


def known(p):
    attr = (ctypes.c_ubyte * 64)()
    rc = hip.hipPointerGetAttributes(attr, ctypes.c_void_p(p))
    hip.hipGetLastError()
    b = bytes(attr)
    sz = ctypes.c_size_t(0)
    rc2 = hip.hipMemPtrGetInfo(ctypes.c_void_p(p), ctypes.byref(sz))
    hip.hipGetLastError()
    return {"attr_rc": rc, "type": int.from_bytes(b[0:4], "little"), "dptr": hex(int.from_bytes(b[8:16], "little")),
            "hptr": hex(int.from_bytes(b[16:24], "little")), "info_rc": rc2, "info_size": sz.value}


def main():
    out = {}
    ctx = engine.Context(0)
    lib = _lib.load()
    for mib in (0.25, 2, 8):
        n = int(mib * (1 << 20))
        a = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8)
        out[f"torch_h2d_{mib}MiB_before"] = known(a.ctypes.data)
        g = torch.from_numpy(a).cuda()
        torch.cuda.synchronize()
        out[f"torch_h2d_{mib}MiB_after"] = known(a.ctypes.data)
        d = torch.empty(n, dtype=torch.uint8)
        d.copy_(g)
        out[f"torch_d2h_{mib}MiB_after"] = known(d.data_ptr())
        b = np.zeros(n, np.uint8)
        engine.read_segments_host(ctx, b, [0], [n], frames_per_seg_cap=16)
        out[f"read_host_{mib}MiB_after"] = known(b.ctypes.data)
        c = np.zeros(n, np.uint8)
        off = np.arange(0, n - 4096, 4096, dtype=np.uint64)
        ln = np.full(off.size, 4096, np.uint32)
        nb = ctypes.c_uint64()
        crc = np.zeros(off.size, np.uint32)
        vp = ctypes.c_void_p
        _lib.check(lib.rh_crc32c_verify_host(ctx.handle, vp(c.ctypes.data), n, vp(off.ctypes.data), vp(ln.ctypes.data),
                                             off.size, vp(crc.ctypes.data), None, ctypes.byref(nb)))
        out[f"verify_host_{mib}MiB_after"] = known(c.ctypes.data)
        _lib.check(lib.rh_synchronize(ctx.handle))
        out[f"verify_host_{mib}MiB_after_ctx_sync"] = known(c.ctypes.data)
        e = np.zeros(n, np.uint8)
        with engine.HostRegistration(ctx, e):
            out[f"register_{mib}MiB_inside"] = known(e.ctypes.data)
        out[f"register_{mib}MiB_after_unregister"] = known(e.ctypes.data)
    torch.cuda.synchronize()
    ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
