mkprof () 
{ 
    tag=$1;
    b=$2;
    title=$3;
    out=$4;
    f=gpurun_out/prof/${tag}_b${b}_timeline.txt;
    { 
        echo "# $title";
        echo;
        echo "rocprofv3 --kernel-trace --stats of \`bench.py --steps 10 --warmup 5 --batch $b $5\` (tools/gpu/prof_bench.sh); one step's kernels in launch order by tools/step_timeline.py.";
        echo;
        echo "$(head -1 $f)";
        echo;
        echo "## Time per kernel family (us per step, launches)";
        echo '```';
        awk 'NR>2{n=$5; sub(/<.*/,"",n); sub(/^_ZN3pca[0-9]+/,"",n); sub(/I.*$/,"",n); t[n]+=$3; c[n]++} END{for(k in t) printf "%8.1f %3d %s\n",t[k],c[k],k}' $f | sort -rn;
        echo '```';
        echo;
        echo "## Step timeline (index, start us, duration us, gap us, kernel)";
        echo '```';
        tail -n +3 $f;
        echo '```'
    } > $out
}
