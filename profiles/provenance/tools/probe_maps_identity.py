"""Probe: does /proc/<pid>/maps name a mapped file by the same dev:inode that stat()
gives?  (overlayfs can show the backing file's device in maps.)  Prints both for a file in
the temp dir, /dev/shm and the repo's gpurun_out/."""
import mmap
import os
import tempfile

for d in (tempfile.gettempdir(), "/dev/shm", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")):
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, f"maps-probe-{os.getpid()}")
    with open(p, "wb") as f:
        f.write(b"\0" * 4096)
    fd = os.open(p, os.O_RDWR)
    m = mmap.mmap(fd, 4096)
    st = os.fstat(fd)
    want = f"{os.major(st.st_dev):02x}:{os.minor(st.st_dev):02x}"
    lines = [l.rstrip() for l in open("/proc/self/maps") if "maps-probe" in l]
    fstype = [l.split()[2] for l in open("/proc/self/mounts") if d.startswith(l.split()[1])]
    print(f"{d}: stat dev {want} ino {st.st_ino}; maps: {lines}; fs candidates {fstype[-1:]}")
    m.close()
    os.close(fd)
    os.unlink(p)
print("uname", os.uname().release)
