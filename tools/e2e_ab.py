"""Full E-RAFT forward (BASELINE config 2) with MIOpen's algorithm search on and off
(profiles/r06u_e2e_kernel_split.txt: no difference; the default stays off).

    python tools/e2e_ab.py [--steps K] [--warmup W]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "e-raft_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--workload", "e2e", "--no-cpu-baseline"] + sys.argv[1:]
    args = bench.parse()
    dev = torch.device("cuda:0")
    for find in (False, True, False):
        torch.backends.cudnn.benchmark = find
        t0 = time.perf_counter()
        res = bench.run_e2e(args, 1, 0, dev, role="workload")
        print(f"cudnn.benchmark={find}: {res['value']} frame-pairs/s, {res['ms_per_step']} ms/step, "
              f"wall {time.perf_counter() - t0:.1f} s, launch {res['config']['launch']}", flush=True)


if __name__ == "__main__":
    main()
