# gnuplot twin of tools/plot.py (the reference's mpi/makePlots.gp:1-40 layout): results/*.txt
# from tools/getAvgs.sh, x = column 3 (ranks), y = column 4 (GB/sec). Reference CUDA constants
# from mpi/CUdata.txt are drawn as dashed lines.
set term postscript eps enhanced color
set style line 1 lt 1 lw 3 lc rgb "red" pt 2
set style line 2 lt 1 lw 3 lc rgb "blue" pt 2
set style line 3 lt 1 lw 3 lc rgb "green" pt 2
set style line 4 lt 2 lw 5 lc rgb "red"
set style line 5 lt 2 lw 5 lc rgb "blue"
set style line 6 lt 2 lw 5 lc rgb "green"
set xlabel "Number of ranks (GPUs)"
set ylabel "Bandwidth (GB/sec)"
set key bottom right
set logscale y
set output "int.eps"
plot "results/INT_MAX.txt" using 3:4 ls 1 title "MI355X Max" with linespoints, \
     "results/INT_MIN.txt" using 3:4 ls 2 title "MI355X Min" with linespoints, \
     "results/INT_SUM.txt" using 3:4 ls 3 title "MI355X Sum" with linespoints, \
     90.8413 ls 4 title "ref CUDA Sum", 90.7905 ls 5 title "ref CUDA Min", 90.7969 ls 6 title "ref CUDA Max"
set output "double.eps"
plot "results/DOUBLE_MAX.txt" using 3:4 ls 1 title "MI355X Max" with linespoints, \
     "results/DOUBLE_MIN.txt" using 3:4 ls 2 title "MI355X Min" with linespoints, \
     "results/DOUBLE_SUM.txt" using 3:4 ls 3 title "MI355X Sum" with linespoints, \
     92.7729 ls 4 title "ref CUDA Sum", 92.6014 ls 5 title "ref CUDA Min", 92.7552 ls 6 title "ref CUDA Max"
