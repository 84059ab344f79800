"""Run tools/libgraph_branch.so's probe inside a torch process (torch's HIP runtime)."""
import ctypes, os
import torch  # noqa: F401
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgraph_branch.so"))
raise SystemExit(lib.probe_main())
