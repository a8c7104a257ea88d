"""Where do a CU-masked stream's workgroups run? (diagnostic build: RAGMI_LIB_AB=<-DRAGMI_DIAG_
BUILD build>). For several masks over the hipExtStreamCreateWithCUMask CU ids, launch 2048
probe workgroups (rag_diag_cu_probe) and report the XCDs (XCC_ID) and distinct (XCD, SE, SH,
CU) slots they ran on. One JSON line per mask."""
import ctypes
import json
import os
import sys
from collections import Counter

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
from ragmi import _lib  # noqa: E402
from ragmi._lib import check  # noqa: E402


def run(L, ids, n_cu=256, n_wg=2048):
    words = (n_cu + 31) // 32
    mask = np.zeros(words, np.uint32)
    for c in ids:
        mask[c // 32] |= np.uint32(1 << (c % 32))
    h = ctypes.c_void_p()
    check(L.rag_stream_create_cu_mask(0, mask.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                      words, ctypes.byref(h)))
    out = torch.full((n_wg, 2), -1, dtype=torch.int32, device="cuda")
    check(L.rag_diag_cu_probe(h, n_wg, ctypes.c_void_p(out.data_ptr())))
    torch.cuda.synchronize()
    L.rag_stream_destroy(h)
    o = out.cpu().numpy()
    xcc = o[:, 0] & 0xF
    hw = o[:, 1].astype(np.uint32)
    cu, sh, se = (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 0x7
    slots = set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
    return {"per_xcc": dict(sorted(Counter(xcc.tolist()).items())), "slots": len(slots),
            "slots_per_xcc": dict(sorted(Counter(s[0] for s in slots).items()))}


def main():
    L = _lib.load()
    n = torch.cuda.get_device_properties(0).multi_processor_count
    masks = {"all": range(n), "ids_0_31": range(32), "ids_0_7": range(8),
             "stride8_from0": range(0, n, 8), "stride32_from31": range(31, n, 32),
             "ids_248_255": range(n - 8, n), "all_but_stride32_from31":
             [c for c in range(n) if c % 32 != 31], "all_but_248_255": range(n - 8)}
    for name, ids in masks.items():
        r = run(L, list(ids), n)
        r.update({"mask": name, "cus_in_mask": len(list(ids))})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
