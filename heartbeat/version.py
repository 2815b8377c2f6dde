"""heartbeat.version (reference heartbeat/version.py)."""
__version__ = "0.1.10"
