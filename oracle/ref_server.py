"""oracle/ref_server.py -- TEST INFRASTRUCTURE ONLY (never part of the product).

The reference's own alignment server (`bowtie2-align-server-s`) and web client
(`bowtie2-align-l`), built from /root/reference by oracle/ref/ into
oracle/_ref, on top of the product's server runner
(bowtie2-server_amd/serve.py: the protocol of BASELINE.md section 3 -- ready
line, <= 10 000 reads per connection, k connections at a time, wall time to
the last `@CO BT2SRV All Done`).  Here `Server` starts the reference server
and `Server.run` uses the reference client unless told otherwise: the stock
baseline and the SAM parity checks of tests/ run the reference end to end.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bowtie2-server_amd"))

import serve  # noqa: E402
from serve import (CHUNK, NATIVE_CLIENT, cgroup_throttled_seconds, dropin_env, free_port,  # noqa: E402,F401
                   host_cpu_seconds, host_cpus, sorted_records, write_fastq_chunks)

REF_DIR = os.path.join(HERE, "_ref")
SERVER = os.path.join(REF_DIR, "bowtie2-align-server-s")
CLIENT = os.path.join(REF_DIR, "bowtie2-align-l")


class Server(serve.Server):
    """serve.Server with the reference server and the reference client as defaults."""

    def __init__(self, index_base, threads=1, args=(), binary=SERVER, **kw):
        super().__init__(index_base, threads=threads, args=args, binary=binary, **kw)

    def run(self, chunk_args, k=1, client=CLIENT, **kw):
        return super().run(chunk_args, k=k, client=client, **kw)
