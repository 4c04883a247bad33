"""MI355X-native batched HTM engine (encoder -> SP -> BacktrackingTM -> anomaly).

Import through the repo-root helper `_pkg.load()` (the package directory name
is not a Python identifier); it registers this package as `rtap_amd`.
"""
from . import _lib
from ._lib import HtmConfig, HtmError, build, default_config
from .engine import HTMEngine
from . import classifier, fleet, harness, ingest
from .harness import AnomalyLikelihood, SLOHarness
from .network import BatchRecordStream, MultiEncoder, Network, ScalarEncoder

__all__ = ["AnomalyLikelihood", "SLOHarness", "HTMEngine", "Network", "BatchRecordStream", "MultiEncoder", "ScalarEncoder", "HtmConfig", "HtmError", "build", "default_config", "_lib"]
