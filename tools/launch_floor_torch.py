"""Run tools/liblaunch_floor.so's probe inside a torch process (torch's HIP runtime)."""
import ctypes, os
import torch  # noqa: F401  (load torch's runtime first)
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblaunch_floor.so"))
raise SystemExit(lib.probe_main())
