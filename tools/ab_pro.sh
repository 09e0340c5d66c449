set -e
timeout -k 10 200 python -u tools/fusedpro_bench.py
for v in 1 2 4 8; do echo "== FQ_PRO_ABL=$v"; FLEXQ_AMD_LIB=tools/libflexq_hip_pa$v.so timeout -k 10 200 python -u tools/fusedpro_bench.py; done
