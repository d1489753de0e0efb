# Scaling plots from tools/getAvgs.sh output (gnuplot >= 5; tools/plot.py is the matplotlib
# equivalent and the one the tests run — gnuplot is not installed in the build image).
#
# Data contract (same columns the reference's mpi/makePlots.gp:21-23 reads): results/<DT>_<OP>.txt,
# column 3 = ranks (GPUs), column 4 = GB/sec. The reference's single-GPU CUDA numbers
# (mpi/CUdata.txt:2-8) are drawn as horizontal reference levels.
#
#   gnuplot tools/makePlots.gp            -> int.eps, double.eps in the current directory

set terminal postscript eps enhanced color font "Helvetica,14" size 6in,4in
set grid ytics lc rgb "#dddddd"
set logscale xy 2
set format y "%g"
set xlabel "GPUs (one rank each)"
set ylabel "GB/s (whole job)"
set key outside right top box

ops = "MAX MIN SUM"
colours = "#d62728 #1f77b4 #2ca02c"

# reference CUDA levels per dtype, in op order SUM MIN MAX (mpi/CUdata.txt)
ref_INT = "90.8413 90.7905 90.7969"
ref_DOUBLE = "92.7729 92.6014 92.7552"

do for [dt in "INT DOUBLE"] {
    set output sprintf("%s.eps", dt eq "INT" ? "int" : "double")
    set title sprintf("%s reductions on MI355X vs the reference's CUDA GPU", dt)
    levels = dt eq "INT" ? ref_INT : ref_DOUBLE
    plot for [i=1:3] sprintf("results/%s_%s.txt", dt, word(ops, i)) using 3:4 \
             with linespoints lw 2 pt 7 lc rgb word(colours, i) title sprintf("MI355X %s", word(ops, i)), \
         for [j=1:3] (real(word(levels, j))) with lines dt 3 lw 2 lc rgb "#555555" \
             title sprintf("reference CUDA %s", word("SUM MIN MAX", j))
}
