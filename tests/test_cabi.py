"""CPU checks of the C-ABI boundary: the library loads without a GPU and exports every
symbol include/td3.h declares, with argument checking that fails loudly."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "td3.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|size_t|void|void\*|double|const char\*)\s*\**\s*(\w+)\s*\(",
                                 txt, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from td3_amd.build import build_library
    build_library()
    from td3_amd import _lib
    return _lib.load()


def test_header_symbols_exported(lib):
    from td3_amd import _lib
    syms = _header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/td3.h but not exported"
        assert s in _lib.SIGNATURES, f"{s} not bound in td3_amd/_lib.py"


def test_no_cpu_fallback_symbols(lib):
    # the product library must not reference the oracle
    data = open(os.path.join(ROOT, "td3_amd", "libtd3hip.so"), "rb").read()
    assert b"td3_oracle" not in data


def test_default_config(lib):
    from td3_amd import _lib
    assert C.sizeof(_lib.td3_config) == lib.td3_config_size()
    cfg = _lib.default_config()
    assert cfg.struct_size == C.sizeof(cfg)
    assert list(cfg.actor_hidden) == [500, 400, 300]      # TD3_featured.py:19
    assert list(cfg.critic_hidden) == [500, 400, 200]     # TD3_featured.py:54
    assert cfg.policy_freq == 2 and abs(cfg.tau - 0.005) < 1e-12
    assert abs(cfg.discount - 0.99) < 1e-12 and abs(cfg.lr - 1e-4) < 1e-15
    assert abs(cfg.policy_noise - 0.2) < 1e-12 and abs(cfg.noise_clip - 0.5) < 1e-12


def test_argument_errors_are_reported(lib):
    from td3_amd import _lib
    h = C.c_void_p()
    assert lib.rb_create(0, 1, 10, 0, 0, C.byref(h)) == -1
    assert b"dims" in lib.td3_last_error()
    cfg = _lib.default_config()
    cfg.state_dim, cfg.action_dim = 17, 40
    assert lib.td3_create(C.byref(cfg), C.byref(h)) == -1
    assert b"action_dim" in lib.td3_last_error()
    with pytest.raises(_lib.TD3Error):
        _lib.check(-1, "x")


def test_config_size_mismatch_is_refused(lib):
    """A binding whose td3_config is shorter than the library's (round 2's INTEGRATION.md stub
    stopped at use_graph) gets -1 and no write past its buffer; a struct_size that is not the
    library's is refused by td3_create before any other field is read."""
    from td3_amd import _lib
    n = lib.td3_config_size()
    buf = (C.c_ubyte * (n + 16))(*([0xAB] * (n + 16)))
    assert lib.td3_default_config(C.cast(buf, C.POINTER(_lib.td3_config)), n - 16) == -1
    assert b"binding out of date" in lib.td3_last_error()
    assert all(b == 0xAB for b in bytes(buf)), "td3_default_config wrote into a mis-sized struct"
    assert lib.td3_default_config(C.cast(buf, C.POINTER(_lib.td3_config)), n) == 0
    assert all(b == 0xAB for b in bytes(buf)[n:]), "td3_default_config wrote past sizeof(td3_config)"
    cfg = _lib.default_config()
    cfg.struct_size = n - 16
    h = C.c_void_p()
    assert lib.td3_create(C.byref(cfg), C.byref(h)) == -1
    assert b"struct_size" in lib.td3_last_error()


def _integration_blocks():
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = txt[txt.index("## The binding a maintainer would add"):]
    return re.findall(r"```python\n(.*?)```", sec, flags=re.S)


def test_integration_snippet(lib, monkeypatch):
    """The binding INTEGRATION.md shows a maintainer, run as written (CPU: struct layout, the
    defaults and td3_create's argument checks; the create / train calls need an MI355X)."""
    from td3_amd import _lib
    blocks = _integration_blocks()
    assert len(blocks) >= 2
    monkeypatch.chdir(ROOT)
    ns = {}
    exec(compile(blocks[0], "INTEGRATION.md", "exec"), ns)
    cfg, td3_config = ns["cfg"], ns["td3_config"]
    assert C.sizeof(td3_config) == C.sizeof(_lib.td3_config) == lib.td3_config_size()
    assert [f[0] for f in td3_config._fields_] == [f[0] for f in _lib.td3_config._fields_]
    assert cfg.struct_size == C.sizeof(td3_config) and cfg.cdq == 1 and cfg.particles == 0
    assert list(cfg.critic_hidden) == [500, 400, 200] and cfg.state_dim == 17
    h = C.c_void_p()
    dl = ns["lib"]
    bad = td3_config.from_buffer_copy(cfg)
    bad.state_dim = 0
    assert dl.td3_create(C.byref(bad), C.byref(h)) == -1
    assert b"dims must be positive" in dl.td3_last_error()
    bad = td3_config.from_buffer_copy(cfg)
    bad.policy_freq = 0
    assert dl.td3_create(C.byref(bad), C.byref(h)) == -1
    assert b"policy_freq" in dl.td3_last_error()


def test_product_modules_import_without_gpu():
    import td3_amd.TD3_featured as tf
    import td3_amd.my_replay_buffer as mrb
    assert tf.TD3 and mrb.ReplayBuffer_featured
