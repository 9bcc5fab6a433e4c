"""Diagnostic: discovery re-walks (rpgpu_job_totals.n_rewalks) and stage
times of one recipe job at several chunk sizes.  Usage:
dbg_discover.py [c1|c2|c5] [nseg] [seg_mib]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import synth
    from redpanda_amd import abi
    from redpanda_amd.engine import Engine
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    nseg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    mib = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    kw = {"c1": synth.C1, "c2": synth.C2, "c5": synth.C5}[which]
    segs = []
    for i in range(nseg):
        a = np.zeros(mib << 20, np.uint8)
        synth.gen_segment(a, i, **kw)
        segs.append(a)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    d = torch.from_numpy(np.concatenate(segs + [np.zeros(256, np.uint8)])).cuda()
    e = Engine(0)
    flags = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
    for chunk in (0, 64 << 10, 1 << 20):
        out = e.alloc_outputs(nseg, int(offs[-1]) // 4096 + 4096, int(offs[-1]) // 64, int(offs[-1]) * 3)
        e.submit(d, offs, out, flags, chunk)
        torch.cuda.synchronize()
        e.set_timing(True)
        for _ in range(3):
            e.submit(d, offs, out, flags, chunk)
        torch.cuda.synchronize()
        tm = e.last_timings()
        e.set_timing(False)
        t = out.totals_host()
        print(f"{which} chunk={chunk >> 10} KiB batches={int(t['n_batches'])} rewalks={int(t['n_rewalks'])} "
              f"discover={tm['discover']:.3f} resolve_plan={tm['resolve_plan']:.3f} total={tm['total']:.3f} ms", flush=True)
        del out
    return 0


if __name__ == "__main__":
    sys.exit(main())
