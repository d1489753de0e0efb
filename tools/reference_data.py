"""The reference's published numbers, as data (no reference file is read or copied at run time).

* ``BGL_VN`` — BlueGene/L virtual-node mode, element-wise ``MPI_Reduce`` of 2 GiB to rank 0, mean
  of the retries per (DATATYPE, OP, ranks) in reduce.c's unit, GiB/s of total data (2^30 B,
  mpi/reduce.c:79,93). Source: mpi/results/{INT,DOUBLE}_{MAX,MIN,SUM}.txt (getAvgs.sh output), the
  series drawn by mpi/makePlots.gp:21-39.
* ``CUDA`` — the single-GPU SDK "kernel 6" constants, GB/s (1e9 B): mpi/CUdata.txt:1-8 (the
  horizontal lines of mpi/makePlots.gp:17-19,29-31).
"""

BGL_VN = {
    ("INT", "MAX"): {64: 8.39020, 256: 44.61860, 1024: 135.86340},
    ("INT", "MIN"): {64: 7.19240, 256: 29.05360, 1024: 116.55080},
    ("INT", "SUM"): {64: 9.18200, 256: 38.64840, 1024: 146.81800},
    ("DOUBLE", "MAX"): {64: 5.60300, 256: 22.52100, 1024: 90.31520},
    ("DOUBLE", "MIN"): {64: 5.49760, 256: 22.12680, 1024: 88.76260},
    ("DOUBLE", "SUM"): {64: 3.81020, 256: 15.31260, 1024: 60.97540},
}

CUDA = {
    ("INT", "SUM"): 90.8413, ("INT", "MIN"): 90.7905, ("INT", "MAX"): 90.7969,
    ("DOUBLE", "SUM"): 92.7729, ("DOUBLE", "MIN"): 92.6014, ("DOUBLE", "MAX"): 92.7552,
}

GIB_PER_GB = 1e9 / 2 ** 30  # a GB/s value times this is GiB/s
