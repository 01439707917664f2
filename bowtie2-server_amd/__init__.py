"""MI355X-native engines for bowtie2's seed-and-extend hot path.

The directory name carries a hyphen, so callers load it by path: the
``bt2g`` module (ctypes binding of include/bt2g.h) and ``tools/bt2_index``
(byte-exact .bt2 index builder for synthetic genomes)."""
