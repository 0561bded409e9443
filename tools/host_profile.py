"""Host-side (Python) profile of the edit loop: cProfile over bench.py's edit at a small frame count,
where the GPU work per launch is small and the host issue rate limits the step time.
usage: python tools/host_profile.py [frames] OUT.txt"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 1
out = sys.argv[2] if len(sys.argv) > 2 else "host_profile.txt"
sys.argv = ["bench.py", "--frames", str(frames), "--steps", "1", "--warmup", "1", "--extras", "none",
            "--no-cpu-baseline", "--no-events"]
import bench  # noqa: E402

pr = cProfile.Profile()
pr.enable()
bench.main()
pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s).sort_stats("tottime")
st.print_stats(45)
st.sort_stats("cumulative").print_stats(45)
open(out, "w").write(s.getvalue())
