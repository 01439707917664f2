"""serve.py -- run an alignment server binary and feed it reads (product side).

The north-star path end to end on one host: a bowtie2 alignment server (the
batch-first server bound to the MI355X engines, integration/bin/
bowtie2-align-server-batch) started on a free port, and the reads sent to it
over the reference's wire protocol by this repository's
multi-connection client, integration/bin/bt2g-client (row (f)-4), or by any
client binary with the reference client's command line:

  * the server is started with the alignment options and `-p threads`, and is
    "ready" once it prints `INFO: Server ready to process`
    (bt2_search.cpp:4898); index load is not timed;
  * reads go out in chunks of <= 10 000 per client connection (the fork's slot
    names make larger connections nondeterministic), k chunks
    in flight at once;
  * wall time runs from the first connection to the end of the last one (a
    connection ends at `@CO BT2SRV All Done`, pat.cpp:2712-2789);
  * SAM records come back with the read names restored by the client
    (pat.cpp:2570-2646); `sorted_records` sorts them for comparison, as the
    reference's own tests do (scripts/sim/Sim.pm:933-947).

Server flags: bt2_search.cpp:543-748 (`--server-port` 679); client port from
BT2CLT_SERVER_PORT (bt2_search.cpp:527-536).  oracle/ref_server.py adds the
reference's own server and client (test infrastructure) on top of this.
"""
import os
import socket
import subprocess
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE_CLIENT = os.path.join(ROOT, "integration", "bin", "bt2g-client")
BATCH_SERVER = os.path.join(ROOT, "integration", "bin", "bowtie2-align-server-batch")
CHUNK = 10_000
CHUNK_MARK = b"@CO BT2G-CLIENT CHUNK "


def dropin_env(index_base, stats_path=None, device=0):
    """Environment of the drop-in server (integration/): the index its engines
    open and where the binding writes its call counts.  (The servers set their
    HIP hardware queues themselves before their first HIP call -- the GPU box
    exports 4; BT2G_HW_QUEUES overrides, default 16: with 32 every kernel of
    the batch server's services ran slower, the 1-mm work queue 6x (r04ae) --
    and the server is started with it too.)"""
    hq = os.environ.get("BT2G_HW_QUEUES", "16")
    env = {"BT2G_INDEX": index_base, "BT2G_DEVICE": str(device), "BT2G_HW_QUEUES": hq, "GPU_MAX_HW_QUEUES": hq}
    if stats_path:
        env["BT2G_ADAPTER_STATS"] = stats_path
    return env


def cgroup_throttled_seconds():
    """Time this container's threads spent throttled by its CPU quota (cgroup
    cpu.stat throttled_usec; nan without a cgroup v2 quota)."""
    try:
        for ln in open("/sys/fs/cgroup/cpu.stat"):
            if ln.startswith("throttled_usec"):
                return int(ln.split()[1]) / 1e6
    except (OSError, ValueError, IndexError):
        pass
    return float("nan")


def host_cpu_seconds():
    """CPU seconds (user + system) this container has spent -- the cgroup's
    cpu.stat (the GPU box's CPU quota is shared by the server, its clients and
    the harness), else the host's /proc/stat."""
    try:
        for ln in open("/sys/fs/cgroup/cpu.stat"):
            if ln.startswith("usage_usec"):
                return int(ln.split()[1]) / 1e6
    except (OSError, ValueError, IndexError):
        pass
    try:
        f = open("/proc/stat").readline().split()
        return (int(f[1]) + int(f[2]) + int(f[3]) + int(f[6]) + int(f[7])) / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, IndexError):
        return float("nan")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def write_fastq_chunks(dirpath, codes, quals, names=None, chunk=CHUNK, codes2=None, quals2=None):
    """FASTQ files of <= chunk reads (pairs: two files per chunk).  Returns a list
    of argument lists for the client (-U f | -1 f1 -2 f2)."""
    acgt = np.frombuffer(b"ACGTN", np.uint8)
    out = []
    n = len(codes)
    for c, lo in enumerate(range(0, n, chunk)):
        hi = min(n, lo + chunk)
        files = []
        for m, (cd, qu) in enumerate(((codes, quals), (codes2, quals2))):
            if cd is None:
                continue
            path = os.path.join(dirpath, f"chunk{c:05d}_{m + 1}.fq")
            with open(path, "wb") as f:
                for i in range(lo, hi):
                    nm = names[i] if names is not None else b"r%d" % i
                    seq = cd[i] if isinstance(cd[i], bytes) else acgt[cd[i]].tobytes()
                    q = qu[i] if isinstance(qu[i], bytes) else np.asarray(qu[i], np.uint8).tobytes()
                    f.write(b"@" + nm + b"\n" + seq + b"\n+\n" + q + b"\n")
            files.append(path)
        out.append(["-U", files[0]] if len(files) == 1 else ["-1", files[0], "-2", files[1]])
    return out


def pinned_cpus():
    """The CPUs the batch server pins itself to ($BT2G_PIN_CPUS, default "auto":
    the first ceil(cgroup quota) CPUs of the affinity mask when the mask is
    larger; integration/bt2g_batch.cpp pin_cpus), or None (no pinning) -- so that
    the stock server can run on the same CPUs."""
    e = os.environ.get("BT2G_PIN_CPUS", "auto")
    if not e or e == "0":
        return None
    n = 0
    if e == "auto":
        try:
            q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
            if q != "max" and int(period) > 0:
                n = -(-int(q) // int(period))
        except (OSError, ValueError):
            n = 0
    else:
        n = int(e)
    mask = sorted(os.sched_getaffinity(0))
    if n <= 0 or len(mask) <= n:
        return None
    return mask[:n]


class Server:
    """One alignment server process on a free port (context manager)."""

    def __init__(self, index_base, threads=1, args=(), binary=BATCH_SERVER, env=None, ready_timeout=600,
                 log_path=None, prefix=(), cpus=None):
        """`prefix`: a launcher put before the server's command line that runs the
        server in its own process (rocprofv3 ... --).  `cpus`: the server process's
        CPU affinity (the stock server on the CPUs the batch server pins itself to)."""
        self.index_base = index_base
        self.port = free_port()
        cmd = list(prefix) + [binary, "-x", index_base, "-p", str(threads), "--server-port", str(self.port)] + list(args)
        self.log_path = log_path or tempfile.mktemp(prefix="bt2srv_", suffix=".log")
        self._log = open(self.log_path, "wb")
        self.proc = subprocess.Popen(cmd, stdout=self._log, stderr=subprocess.STDOUT,
                                     env=dict(os.environ, **(env or {})),
                                     preexec_fn=(lambda: os.sched_setaffinity(0, cpus)) if cpus else None)
        t0 = time.time()
        while True:
            txt = open(self.log_path, "rb").read()
            if b"Server ready to process" in txt and b"Server listening" in txt:
                break
            if self.proc.poll() is not None:
                raise RuntimeError(f"server exited rc={self.proc.returncode}: {txt[-2000:].decode(errors='replace')}")
            if time.time() - t0 > ready_timeout:
                self.close()
                raise TimeoutError("server not ready")
            time.sleep(0.05)
        self.load_s = time.time() - t0

    def log(self):
        return open(self.log_path, "rb").read().decode(errors="replace")

    def run(self, chunk_args, k=1, client=NATIVE_CLIENT, timeout=1200, warmup=(), keep=True):
        """Send every chunk (client argument lists) over at most k concurrent
        connections.  Returns (wall seconds, list of SAM texts in chunk order).
        `client`: NATIVE_CLIENT (one bt2g-client process for all the chunks, k
        connections at a time) or the path of a client with the reference
        client's command line (one process per chunk, k at a time).
        `warmup`: chunks sent first, untimed, output dropped (a long-running
        server past its start-up: workers spawned, per-worker state allocated).
        `keep=False` (native client only): the SAM still comes back over every
        connection and through the client's stdout, but is not split per chunk
        here (outs is None); the client counts the aligned reads itself
        (--count-aligned, in self.last_aligned) -- the harness's own counting
        in Python (~1 s per 1 M reads) stays out of the timed passes."""
        if warmup:
            self.run(list(warmup), k=min(k, len(warmup)), client=client, timeout=timeout)
        outs = [None] * len(chunk_args)
        errs = []
        self.last_aligned = None
        nxt = [0]
        lock = threading.Lock()
        env = dict(os.environ, BT2CLT_SERVER_PORT=str(self.port), BT2CLT_SERVER_HOST="127.0.0.1")

        def worker():
            while True:
                with lock:
                    i = nxt[0]
                    nxt[0] += 1
                if i >= len(chunk_args):
                    return
                r = subprocess.run([client, "-x", self.index_base, "--no-hd"] + chunk_args[i], env=env,
                                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout)
                if r.returncode != 0:
                    errs.append((i, r.returncode, r.stderr[-2000:]))
                outs[i] = r.stdout

        def native():
            if any(not (len(a) == 2 and a[0] == "-U") and not (len(a) == 4 and a[0] == "-1" and a[2] == "-2")
                   for a in chunk_args):
                # other inputs (-f, --tab6, ...): one client process per chunk, in turn
                tot = 0
                for i, a in enumerate(chunk_args):
                    r = subprocess.run([client, "-x", self.index_base, "--no-hd", "--count-aligned"] + list(a),
                                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout)
                    if r.returncode != 0:
                        errs.append((i, r.returncode, r.stderr[-2000:]))
                        return
                    for ln in r.stderr.splitlines():
                        if ln.startswith(b"bt2g-client: aligned "):
                            tot += int(ln.split()[2])
                    outs[i] = r.stdout
                self.last_aligned = tot
                return
            lst = tempfile.mktemp(prefix="bt2g_chunks_", suffix=".txt")
            with open(lst, "w") as f:
                for a in chunk_args:
                    if a[0] == "-U":
                        f.write(f"U {a[1]}\n")
                    elif a[0] == "-1" and a[2] == "-2" and len(a) == 4:
                        f.write(f"P {a[1]} {a[3]}\n")
                    else:
                        raise ValueError(f"chunk arguments not supported by the native client: {a}")
            r = subprocess.run([client, "-x", self.index_base, "--chunks", lst, "-k", str(max(1, k)),
                                "--mark-chunks", "--count-aligned"], env=env, stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, timeout=timeout)
            os.unlink(lst)
            if r.returncode != 0:
                errs.append((-1, r.returncode, r.stderr[-2000:]))
                return
            for ln in r.stderr.splitlines():
                if ln.startswith(b"bt2g-client: aligned "):
                    self.last_aligned = int(ln.split()[2])
            if not keep:
                return
            parts = r.stdout.split(CHUNK_MARK)
            for p in parts[1:]:
                nl = p.index(b"\n")
                outs[int(p[:nl])] = p[nl + 1:]

        import resource
        ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        c0 = self.cpu_seconds()
        h0 = host_cpu_seconds()
        th0 = cgroup_throttled_seconds()
        t0 = time.perf_counter()
        if os.path.basename(client) == os.path.basename(NATIVE_CLIENT):
            native()
        else:
            ths = [threading.Thread(target=worker) for _ in range(max(1, min(k, len(chunk_args))))]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        dt = time.perf_counter() - t0
        self.last_cpu_s = self.cpu_seconds() - c0        # server CPU time (all threads) over the run
        ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        # the clients' CPU time (the client processes of this run, reaped)
        self.last_client_cpu_s = (ru1.ru_utime + ru1.ru_stime) - (ru0.ru_utime + ru0.ru_stime)
        self.last_host_cpu_s = host_cpu_seconds() - h0   # every process of the host (clients included)
        self.last_throttled_s = cgroup_throttled_seconds() - th0
        self.last_rss_gb = self.rss_gb()
        self.last_threads = self.thread_cpu()
        if errs:
            # the server's own output (kept in its log file, which outlives the
            # server): why a connection failed is usually there, not in the client's
            raise RuntimeError(f"client failures: {errs[:3]}\nserver rc={self.proc.poll()} "
                               f"(log {self.log_path}), tail:\n{self.log()[-4000:]}")
        if not keep and os.path.basename(client) == os.path.basename(NATIVE_CLIENT):
            if self.last_aligned is None:
                raise RuntimeError("the client reported no aligned count")
            return dt, None
        if any(o is None for o in outs):
            raise RuntimeError("a chunk came back without output")
        return dt, outs

    def thread_cpu(self):
        """{thread name: [threads, CPU seconds, busiest thread's CPU seconds]} of the server."""
        out = {}
        tck = os.sysconf("SC_CLK_TCK")
        try:
            tids = os.listdir(f"/proc/{self.proc.pid}/task")
        except OSError:
            return out
        for t in tids:
            try:
                txt = open(f"/proc/{self.proc.pid}/task/{t}/stat").read()
            except OSError:
                continue
            name = txt[txt.index("(") + 1:txt.rindex(")")]
            f = txt.rsplit(")", 1)[1].split()
            cs = (int(f[11]) + int(f[12])) / tck
            e = out.setdefault(name, [0, 0.0, 0.0])
            e[0] += 1
            e[1] += cs
            e[2] = max(e[2], cs)
        return out

    def smaps_top(self, k=6):
        """The server's largest mappings by resident size (MB, with the part in
        transparent huge pages): where its memory is."""
        rows, cur = [], None
        try:
            for ln in open(f"/proc/{self.proc.pid}/smaps"):
                f = ln.split()
                if not f:
                    continue
                if "-" in f[0] and not f[0].endswith(":"):
                    cur = {"range": f[0], "name": f[5] if len(f) > 5 else "", "rss_mb": 0.0, "thp_mb": 0.0}
                    rows.append(cur)
                elif f[0] == "Rss:" and cur is not None:
                    cur["rss_mb"] = int(f[1]) / 1024
                elif f[0] == "AnonHugePages:" and cur is not None:
                    cur["thp_mb"] = int(f[1]) / 1024
        except (OSError, ValueError):
            return []
        rows.sort(key=lambda r: -r["rss_mb"])
        return rows[:k]

    def rss_gb(self):
        """Resident memory of the server (GB)."""
        try:
            for ln in open(f"/proc/{self.proc.pid}/status"):
                if ln.startswith("VmRSS:"):
                    return int(ln.split()[1]) / 1e6
        except (OSError, ValueError):
            pass
        return float("nan")

    def cpu_seconds(self):
        """User + system CPU seconds of the server process so far (/proc/<pid>/stat)."""
        try:
            f = open(f"/proc/{self.proc.pid}/stat").read().rsplit(")", 1)[1].split()
            return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")
        except (OSError, ValueError, IndexError):
            return float("nan")

    def close(self):
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=20)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        self._log.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def sorted_records(sam_texts):
    """SAM alignment records (no header / @CO lines), sorted."""
    recs = []
    for t in sam_texts:
        for ln in t.split(b"\n"):
            if ln and not ln.startswith(b"@"):
                recs.append(ln)
    recs.sort()
    return recs


def host_cpus():
    """CPU budget of this host/job: nproc, scheduler affinity, cgroup quota, model."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = int(subprocess.run(["nproc"], stdout=subprocess.PIPE).stdout or 0)
    usable = int(quota) if quota else aff
    usable = max(1, min(usable, aff, nproc or aff))
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "usable": usable, "model": model}
