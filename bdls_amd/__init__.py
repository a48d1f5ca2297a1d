"""bdls_amd -- MI355X-native batched ECDSA verification for the BDLS / Fabric
signature-verification hot path (BCCSP Verify). See DESIGN.md."""
from ._lib import EngineError, LIB_PATH  # noqa: F401

__version__ = "0.1.0"
