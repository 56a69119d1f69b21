// (all include/orbx.h entry points are implemented; file kept empty)
