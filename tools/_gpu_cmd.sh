export TMPDIR=/tmp
timeout -k 10 1000 python tools/ab.py 3 default prev nordiv nofdiv neither -- --steps 48 --warmup 4
