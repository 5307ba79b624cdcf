"""Print the top entries of a cProfile dump (cumulative and own time).
usage: prof_top.py FILE [N]"""
import pstats
import sys

st = pstats.Stats(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
st.sort_stats('cumulative').print_stats(n)
st.sort_stats('tottime').print_stats(n)
