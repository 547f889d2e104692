"""Probe: which hardware queue does each kind of HIP stream get?

Run under ``rocprofv3 --kernel-trace`` and read Queue_Id per kernel:
eight normal-priority torch streams first (more than GPU_MAX_HW_QUEUES=4),
then a greatest-priority stream and a CU-masked stream (all CUs, and half
of them).  Each stream launches one tagged fill (tensor.fill_ of a size
that names the stream) so the trace rows can be matched: the fill of
stream k writes 4096 * (k + 1) elements.  Prints the tag map.
"""
import ctypes as C
import json

import torch

dev = torch.device("cuda:0")
hip = C.CDLL("libamdhip64.so")
ncu = torch.cuda.get_device_properties(dev).multi_processor_count


def masked_stream(mask_cus):
    words = (ncu + 31) // 32
    m = (C.c_uint32 * words)()
    for cu in mask_cus:
        m[cu // 32] |= 1 << (cu % 32)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(words), m)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


streams = [("normal%d" % k, torch.cuda.Stream(device=dev)) for k in range(8)]
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
streams.append(("prio_greatest", torch.cuda.Stream(device=dev, priority=-1)))
streams.append(("prio_greatest2", torch.cuda.Stream(device=dev, priority=-1)))
streams.append(("cumask_all", masked_stream(range(ncu))))
streams.append(("cumask_half", masked_stream(range(0, ncu, 2))))
streams.append(("cumask_all2", masked_stream(range(ncu))))
tags = {}
bufs = []
for k, (name, s) in enumerate(streams):
    n = 4096 * (k + 1)
    t = torch.empty(n, dtype=torch.float32, device=dev)
    with torch.cuda.stream(s):
        for _ in range(3):
            t.fill_(float(k))
    bufs.append(t)
    tags[name] = n
torch.cuda.synchronize()
print(json.dumps({"cus": ncu, "tags_elements": tags}))
