"""sailrecon_amd — MI355X-native SailRecon aggregator + camera-pose head.

Mirrors the reference package layout (sailrecon.models / heads / layers / utils) and
state_dict names; every hot-path op runs in libsfm_amd.so (hand-written gfx950 HIP).
"""

__version__ = "0.1.0"
