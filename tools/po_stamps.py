"""Diagnostics: phase cycles of k_ba_pose_only (frame 0, thread 0) from a LORB_PO_STAMPS build
(tools/build_variant.sh post -DLORB_PO_STAMPS; run with LORB_LIB_PATH=variants/liblorb_post.so).
Tags: 0 entry, 1 linearisation pass start, 2 its sums done, 3 wave reduction done, 4 barrier done,
5 step solved (candidate pass start), 6 candidate sums done, 7 barrier done, 8 exit."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lorb_slam_amd import synth  # noqa: E402
from lorb_slam_amd.runtime import Context, lib  # noqa: E402

ctx = Context(0)
L = lib()
for rep in range(3):
    pb = synth.pose_only_batch(seed=rep, n_frames=1, n_res=200)
    ctx.ba_pose_only(pb)
    buf = (C.c_ulonglong * 64)()
    assert L.lorb_debug_po_stamps(buf) == 0
    st = np.frombuffer(buf, np.uint64).reshape(32, 2).astype(np.int64)
    n = int(np.argmax(st[:, 0] == 0)) if (st[:, 0] == 0).any() else 32
    t0 = st[0, 0]
    print("call", rep, " ".join("%d:%d" % (st[i, 1], st[i, 0] - (st[i - 1, 0] if i else t0)) for i in range(n)))
