mkdir -p gpurun_out/psnr5
bash scripts/psnr.sh list gpurun_out/psnr5 oracle 780 250,251,252,253,254,256,257,258 259,260,261,262,291,292,293,294 296,297,298,300,302,304,333,335 336,337,339,340,341,344,345,346 > gpurun_out/psnr5/list.out 2>&1 &
p1=$!
bash scripts/psnr.sh pairs gpurun_out/psnr5 347 20 6 780 fp32 oracle > gpurun_out/psnr5/pairs.out 2>&1
r2=$?
wait $p1; r1=$?
cat gpurun_out/psnr5/list.out gpurun_out/psnr5/pairs.out
echo "list rc=$r1 pairs rc=$r2"
[ $r1 -eq 0 ] && [ $r2 -eq 0 ]
