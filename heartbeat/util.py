"""heartbeat.util (reference heartbeat/util.py:30-96): base64 helpers and the
GPU-evaluated KeyedPRF of heartbeat_amd.util."""
from heartbeat_amd.util import KeyedPRF, hb_decode, hb_encode  # NOQA

__all__ = ["hb_encode", "hb_decode", "KeyedPRF"]
