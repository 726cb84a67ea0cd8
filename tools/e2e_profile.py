"""cProfile of bench.py's end-to-end train_on_policy leg (ppo.yaml variant, 3
generations after the warm-up): where the host time of the selection /
regrouping / mutation phases goes.  Prints the top functions by cumulative
and by own time (diagnostic)."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py"]
os.environ.setdefault("AGX_BENCH_E2E_LONG", "0")
import bench  # noqa: E402

if __name__ == "__main__":
    pr = cProfile.Profile()
    orig = bench.train_on_policy_leg

    pr.enable()
    out = orig(generations=int(os.environ.get("GENS", 3)))
    pr.disable()
    print(out, file=sys.stderr)
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
        print(s.getvalue())
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s).sort_stats("tottime")
    for pat in os.environ.get("CALLERS", "'sum' of|zeros_like|_generate|'item' of|_train_stream").split("|"):
        st.print_callers(pat)
    for pat in os.environ.get("CALLEES", "regroup|clone_states|gather_records|_clone_host_attributes|select").split("|"):
        st.print_callees(pat)
    print(s.getvalue())
