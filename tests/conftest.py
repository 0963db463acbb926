"""Shared fixtures.  `-m "not gpu"` runs on CPU; `-m gpu` needs an MI355X."""
from __future__ import annotations

import gzip
import json
import os
import sys
from pathlib import Path

# The production configuration (bench.py, the CLI): 8 HIP hardware queues, so the library runs six
# workspace slots on streams that do not share queues.  Read when HIP starts, so set before any test
# touches the GPU.  RT_HW_QUEUES overrides; a GPU_MAX_HW_QUEUES already in the environment is kept
# (test_gpu_slots.py runs the slot/arena tests at HIP's default of 4 queues in a child process).
if os.environ.get("RT_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["RT_HW_QUEUES"]
else:
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import __graft_entry__ as graft  # noqa: E402

GOLDEN_DIR = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def pkg():
    # Import torch first so librt_hip.so binds to the same HIP runtime
    # (libamdhip64.so.7) that torch's device buffers and streams come from.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    return graft.import_pkg()


@pytest.fixture(scope="session")
def oracle():
    return graft.import_oracle()


@pytest.fixture(scope="session")
def goldens():
    return json.loads((GOLDEN_DIR / "goldens.json").read_text())["goldens"]


def golden_by_name(goldens, name):
    for g in goldens:
        if g["name"] == name:
            return g
    raise KeyError(name)


def load_golden_image(cam: dict) -> np.ndarray:
    with gzip.open(GOLDEN_DIR / cam["file"], "rb") as f:
        data = f.read()
    return np.frombuffer(data, dtype=np.uint8).reshape(cam["height"], cam["width"], 3)


@pytest.fixture(scope="session")
def scene_dir(tmp_path_factory, pkg):
    """All golden configs written as XML files (derived scenes included)."""
    d = tmp_path_factory.mktemp("scenes")
    names = ["C1_simple", "C2_cornellbox_800_d0", "hm_verbatim", "C3_hm_1080p_d6", "C5_hm_8k_d6"]
    for f in sorted((GOLDEN_DIR / "scenes").glob("*.xml.gz")):
        names.append(f.name[:-3])
    for n in names:
        pkg.scenes.write_config(n, d)
    return d


def config_path(scene_dir: Path, config: str) -> Path:
    return scene_dir / (config if config.endswith(".xml") else config + ".xml")
