#!/usr/bin/env python3
"""Engine-path GraphSAGE (runner, PPI schema) with a watchdog: dumps every thread's stack
and exits if a run makes no progress for 60 s.  Usage: engine_hang_probe.py [runner flags]"""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from euler_amd.tools.runner import main as run

    faulthandler.dump_traceback_later(60, exit=True)
    t = time.time()
    base = ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "256", "--total_step", "150", "--log_steps",
            "10", "--device", "cuda", "--seed", "3", "--fanouts", "5", "3", "--learning_rate", "0.01",
            "--model_dir", "/tmp/engine_hang_probe_%d" % os.getpid()]
    r = run(base + sys.argv[1:], model="graphsage")
    print("done", r, round(time.time() - t, 1), flush=True)


if __name__ == "__main__":
    main()
