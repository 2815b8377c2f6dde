"""heartbeat.exc (reference heartbeat/exc.py:29-35): the one exception class
the library raises, defined in heartbeat_amd.exc."""
from heartbeat_amd.exc import HeartbeatError  # NOQA

__all__ = ["HeartbeatError"]
