"""Host-side profile of the Wide&Deep PS bench step (cProfile, top functions)."""
import cProfile
import pstats
import sys
import types

sys.argv = ['bench.py', '--model', 'wdl', '--steps', '60', '--warmup', '10']
import bench  # noqa: E402

pr = cProfile.Profile()
pr.enable()
bench.main()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats('cumulative').print_stats(35)
st.sort_stats('tottime').print_stats(25)
