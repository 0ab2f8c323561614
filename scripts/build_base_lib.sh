# Build the committed tree's library into abtmp/base.so (the "A" of an A/B run;
# bench.py loads it with TPF_LIB=abtmp/base.so).  Leaves the working tree as it was.
set -e
cd "$(dirname "$0")/.."
rm -rf /tmp/tpf_base && mkdir -p /tmp/tpf_base abtmp
git archive HEAD turbopfor-cpp_amd include | tar -x -C /tmp/tpf_base
make -s -C /tmp/tpf_base/turbopfor-cpp_amd -j8
cp /tmp/tpf_base/turbopfor-cpp_amd/lib/libturbopfor_amd.so abtmp/base.so
echo "abtmp/base.so <- $(git rev-parse --short HEAD)"
