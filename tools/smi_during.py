#!/usr/bin/env python3
"""Sample the GPU's clocks and power with rocm-smi while a command runs.

    python tools/smi_during.py OUT.jsonl -- CMD ...

Starts CMD as a child process (this process never touches the GPU), writes
one JSON line per rocm-smi sample (every ~0.5 s) to OUT.jsonl until the child
exits, and exits with the child's code."""
import json
import subprocess
import sys
import time


def main() -> int:
    out = sys.argv[1]
    cmd = sys.argv[sys.argv.index("--") + 1:]
    child = subprocess.Popen(cmd)
    t0 = time.time()
    with open(out, "w") as f:
        while child.poll() is None:
            try:
                r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--json"], capture_output=True,
                                   text=True, timeout=10)
                rec = {"t": round(time.time() - t0, 2), "smi": json.loads(r.stdout) if r.stdout.strip() else None}
            except (OSError, subprocess.SubprocessError, ValueError) as e:
                rec = {"t": round(time.time() - t0, 2), "error": str(e)}
            f.write(json.dumps(rec) + "\n")
            f.flush()
            time.sleep(0.5)
    return child.wait()


if __name__ == "__main__":
    sys.exit(main())
