"""td3_amd -- MI355X-native TD3 gradient step (replay sample + TD3.train) for gfx950.

Modules mirror the reference's import surface (/root/reference, main.py:203-208):

    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured as ReplayBuffer

All compute runs in libtd3hip.so (hand-written HIP kernels, C-ABI in include/td3.h);
there is no CPU fallback.
"""
__version__ = "0.1.0"
