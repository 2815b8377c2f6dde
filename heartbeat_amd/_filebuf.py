"""Turn the reference's duck-typed file objects (read/seek/tell,
README.md:13) into one contiguous host buffer without copying when possible:
BytesIO -> its buffer, real files -> a read-only mmap, anything else -> read().
The buffer starts at the file's current position, as PySwizzle's reads do
(PySwizzle.py:299)."""
import io
import mmap
import os

import numpy as np


class FileBuffer(object):
    def __init__(self, file):
        self._mm = None
        self.file = file
        start = 0
        try:
            start = file.tell()
        except Exception:
            start = 0
        self.start = start
        arr = None
        if isinstance(file, io.BytesIO):
            arr = np.frombuffer(file.getbuffer(), dtype=np.uint8)[start:]
        elif isinstance(file, (bytes, bytearray, memoryview)):
            arr = np.frombuffer(file, dtype=np.uint8)
        else:
            fd = None
            try:
                fd = file.fileno()
            except Exception:
                fd = None
            if fd is not None:
                try:
                    size = os.fstat(fd).st_size
                    if size > start:
                        self._mm = mmap.mmap(fd, 0, access=mmap.ACCESS_READ)
                        arr = np.frombuffer(self._mm, dtype=np.uint8)[start:]
                    else:
                        arr = np.zeros(0, dtype=np.uint8)
                except (OSError, ValueError):
                    arr = None
            if arr is None:
                data = file.read()
                if isinstance(data, str):
                    data = data.encode("latin-1")
                arr = np.frombuffer(bytes(data), dtype=np.uint8)
                self.start = None   # already consumed
        self.arr = arr
        self.len = int(arr.shape[0])

    @property
    def addr(self):
        return self.arr.ctypes.data if self.len else None

    def consume(self):
        """Leave the file at end of file, as the reference's reads do."""
        if self.start is not None:
            try:
                self.file.seek(self.start + self.len)
            except Exception:
                pass

    def close(self):
        self.arr = None
        if self._mm is not None:
            try:
                self._mm.close()
            except BufferError:
                pass
            self._mm = None
