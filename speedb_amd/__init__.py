"""speedb_amd -- MI355X-native block-checksum engine for Speedb's per-block
CRC32C / XXH3 compute-and-verify path (SST block trailers, WAL records).

The hot path is hand-written HIP for gfx950 (speedb_amd/csrc), exported as a
C ABI (include/speedb_amd/mck.h) and built in-tree into
speedb_amd/libspeedb_amd.so.  Importing this package without that library
raises ImportError: there is no CPU fallback.
"""
import torch  # noqa: F401  (torch's HIP runtime is mapped before the engine's dlopen, as the tests do)
from . import _lib  # noqa: F401  (fails loudly if the engine is not built)
from .checksum import *  # noqa: F401,F403
from .checksum import __all__ as _checksum_all
from . import sst  # noqa: F401  (whole-SST-file verification)
from . import blob  # noqa: F401  (blob file records)
from . import block  # noqa: F401  (per-KV protection of block entries)
from . import handoff  # noqa: F401  (WritableFileWriter checksum handoff)

__all__ = list(_checksum_all)
__version__ = "0.1.0"
