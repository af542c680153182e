"""Run a command as a child process; print its wall time and peak RSS (MiB) to stderr."""
import resource
import subprocess
import sys
import time

t = time.time()
rc = subprocess.call(sys.argv[1:])
print(f"[timed] rc {rc} wall_s {time.time() - t:.1f} maxrss_mib {resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss / 1024:.0f}",
      file=sys.stderr, flush=True)
sys.exit(rc)
