import sys, os
os.environ["CYC_SEGV_TRACE"] = "1"
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import test_gpu_parity as t
for i in range(int(sys.argv[1])):
    t.test_graph_and_eager_paths_agree(0)
    print("iter", i, "ok", flush=True)
