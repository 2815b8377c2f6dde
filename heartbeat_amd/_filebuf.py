"""Turn the reference's duck-typed file objects (read/seek/tell,
README.md:13) into one contiguous host buffer without copying when possible:
BytesIO -> its buffer, real files -> a read-only mmap, anything else -> read().

Two views, matching the two ways the reference touches the file:

* encode (``from_start=False``): the buffer starts at the file's CURRENT
  position, as PySwizzle.encode's sequential ``file.read(sectorsize)`` calls do
  (PySwizzle.py:299; cxx PythonSeekableFile::read, PythonSeekableFile.hxx:47-54);
  ``consume()`` then leaves the file at EOF like those reads.
* prove (``from_start=True``): the buffer is the WHOLE file from offset 0,
  because prove seeks ABSOLUTE offsets ``index*chunk_size + j*sectorsize``
  before every read (PySwizzle.py:353-355; cxx shacham_waters_private.cxx:
  762-764), whatever the position the caller left the file at.  ``restore()``
  puts the caller's position back (the reference leaves the file wherever its
  last read ended; callers must not rely on either).

A read()-only object without ``seek`` cannot be rewound: it is read from its
current position in both views (the reference's prove would fail on it with
an AttributeError on ``seek``).

Short reads.  The reference reads ``file.read(sectorsize)`` per sector and
stops the encode at the FIRST read that returns fewer than ``sectorsize``
bytes (PySwizzle.py:299-306; prove: :355-360), treating it as end of file.
For seekable files, BytesIO and any blocking file object that returns short
reads only at EOF, that is exactly "the bytes up to EOF", which is what the
buffer here holds.  An object that returns short reads MID-stream (an
unbuffered socket, a raw pipe, an io.RawIOBase reader) makes the reference
truncate the tags at the first short read -- at a point that depends on the
sizes its reads happened to return, not on the data -- while the fallback
below reads such an object to EOF with one ``read()`` and tags all of it.
Wrap such streams in ``io.BufferedReader`` (or read them into a BytesIO)
first if the reference's truncation is wanted; INTEGRATION.md section 6.
"""
import io
import mmap
import os

import numpy as np


class FileBuffer(object):
    def __init__(self, file, from_start=False, populate=True):
        self._mm = None
        self.file = file
        self.from_start = from_start
        pos = 0
        try:
            pos = file.tell()
        except Exception:
            pos = 0
        self.pos = pos                       # caller's position, for restore()
        start = 0 if from_start else pos
        self.start = start
        arr = None
        # where the bytes live: "bytesio" / "bytes" (the caller's buffer),
        # "mmap" (a read-only mapping of a real file), "read" (one read() copy)
        self.kind = "read"
        if isinstance(file, io.BytesIO):
            arr = np.frombuffer(file.getbuffer(), dtype=np.uint8)[start:]
            self.kind = "bytesio"
        elif isinstance(file, (bytes, bytearray, memoryview)):
            arr = np.frombuffer(file, dtype=np.uint8)
            self.kind = "bytes"
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
                        # encode reads every byte: prefault the mapping
                        # (MAP_POPULATE) instead of taking page faults inside
                        # the staging copies -- unless the encode page-locks
                        # the bytes itself (populate=False: the registration
                        # faults them in, overlapped with the copies); prove
                        # reads only the challenged blocks and maps lazily
                        flags = mmap.MAP_SHARED
                        if not from_start and populate and hasattr(mmap, "MAP_POPULATE"):
                            flags |= mmap.MAP_POPULATE
                        self._mm = mmap.mmap(fd, 0, flags=flags, prot=mmap.PROT_READ)
                        arr = np.frombuffer(self._mm, dtype=np.uint8)[start:]
                        self.kind = "mmap"
                    else:
                        arr = np.zeros(0, dtype=np.uint8)
                except (OSError, ValueError):
                    arr = None
            if arr is None:
                # a file-like object without a usable fd: one read() to EOF
                # (see "Short reads" above for how this differs from the
                # reference on streams that return short reads mid-stream)
                if from_start:
                    try:
                        file.seek(0)
                    except Exception:
                        pass
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

    def restore(self):
        """Put the caller's file position back."""
        try:
            self.file.seek(self.pos)
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
