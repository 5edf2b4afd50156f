"""Shared fixtures. `gpu`-marked tests need a real MI355X (run via gpurun);
everything else runs on the CPU-only container."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "neuronabox-nccl_amd")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu on the GPU box")


# Run order of the GPU suite: the single-GPU parity core first —
# every type x op vs the oracle, config B at full size, config A, the API
# entry points, config C — then the multi-process transport and the stress
# files, so that `-x` can never hide the core oracle checks behind a
# transport failure. Tests inside a file keep their order; files not listed
# run between the core and the transport group.
GPU_FILE_ORDER = [
    "test_reduce_gpu.py", "test_config_a.py", "test_nccl_api_gpu.py", "test_rccl_corroboration_gpu.py",
    "test_sched_stress_gpu.py", "test_c_perf_gpu.py", "test_bench_rccl_gpu.py",
    None,   # everything else
    "test_configs_gpu.py", "test_clique_transport_gpu.py", "test_multiprocess_gpu.py",
    "test_multiprocess_churn_gpu.py", "test_multiprocess_stress_gpu.py",
]


def gpu_order_key(item_path: str, test_name: str = "") -> tuple:
    base = os.path.basename(item_path)
    rank = GPU_FILE_ORDER.index(base) if base in GPU_FILE_ORDER else GPU_FILE_ORDER.index(None)
    # test_configs_gpu.py: config C (one GPU) before configs D / E (8 ranks)
    sub = 1 if base == "test_configs_gpu.py" and "8_ranks" in test_name else 0
    if base == "test_configs_gpu.py" and not sub:
        rank = GPU_FILE_ORDER.index("test_bench_rccl_gpu.py")
    return (rank, sub)


def pytest_collection_modifyitems(session, config, items):
    if os.environ.get("NBX_GPU_TEST_ORDER") == "files":   # collection order (replays an earlier run's order)
        return
    keyed = [(gpu_order_key(str(it.fspath), it.name), i, it) for i, it in enumerate(items)]
    keyed.sort(key=lambda t: (t[0], t[1]))
    items[:] = [t[2] for t in keyed]


def load_package():
    """Import neuronabox-nccl_amd (hyphenated directory) as `neuronabox_nccl_amd`."""
    name = "neuronabox_nccl_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def nbx():
    return load_package()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch
