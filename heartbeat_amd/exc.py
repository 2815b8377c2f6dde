"""HeartbeatError, as in the reference (heartbeat/exc.py:29-35): a single
exception type carrying ``.message``; ``str(e)`` is the message."""


class HeartbeatError(Exception):

    def __init__(self, message):
        Exception.__init__(self, message)
        self.message = message

    def __str__(self):
        return self.message


# the reference's module path (heartbeat/exc.py): pickles and tracebacks name
# heartbeat.exc, which re-exports this class (the repo's heartbeat/ package)
HeartbeatError.__module__ = "heartbeat.exc"
