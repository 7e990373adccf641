"""The host-to-host leg of bench.py alone (for rocprofv3 --kernel-trace --memory-copy-trace and
VH_PIPE_TRACE runs): n = batches x 256 heterogeneous studies streamed through vh_pipe.

  python3 scripts/h2h_leg.py [--slots 3] [--sub 224] [--batches 12] [--keep-batch]

--keep-batch also holds a 256-study device batch (and its stream) open, as bench.py did in
round 3 while it measured this leg."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--sub", type=int, default=224)
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--keep-batch", action="store_true")
    ap.add_argument("--unaligned", action="store_true", help="plain np.empty host arrays")
    ap.add_argument("--torch", action="store_true", help="initialise torch's HIP context first (as bench.py does)")
    ap.add_argument("--warm-device", type=int, default=0,
                    help="run this many 256-study device-resident steps first (as bench.py does)")
    ap.add_argument("--cpu-load", type=float, default=0.0,
                    help="run bench.py's CPU baseline for this many seconds first")
    a = ap.parse_args()
    if a.cpu_load > 0:
        bench.cpu_baseline(128, 128, 24, seconds=a.cpu_load)
    if a.torch:
        import torch
        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    from vent_analysis_amd import _lib
    R, C, Z, nb = 128, 128, 24, 256
    Bt = _lib.Batch(R, C, Z, nb) if (a.keep_batch or a.warm_device) else None
    if a.warm_device:
        from vent_analysis_amd.synth import synth_batch
        hw, mw = synth_batch(R, C, Z, nb, base_seed=0, unique=64, vary=True)
        Bt.upload(hw, mw)
        o = _lib.Batch.options(do_n4=True, vox=(1.5, 1.5, 10.0), do_cohort=True)
        for _ in range(a.warm_device):
            Bt.run(o)
        Bt.sync()
        if not a.keep_batch:
            Bt.close()
            Bt = None
    opts = _lib.Batch.options(do_n4=True, vox=(1.5, 1.5, 10.0), do_cohort=True, profile=False)
    args = argparse.Namespace(h2h_slots=a.slots, h2h_sub=a.sub, h2h_batches=a.batches)
    h = bench.host_to_host(R, C, Z, nb, args, 0, opts, 500, aligned=not a.unaligned)
    h["vol_s"] = round(h["volumes"] / h["seconds"], 1)
    h["keep_batch"] = a.keep_batch
    h["aligned"] = not a.unaligned
    h["torch"] = a.torch
    h["warm_device"] = a.warm_device
    h["cpu_load"] = a.cpu_load
    h["d2h_late"] = os.environ.get("VH_PIPE_D2H_LATE", "0")
    print(json.dumps(h), flush=True)
    if Bt:
        Bt.close()


if __name__ == "__main__":
    main()
