// lsg_serial_pair_wide.hip -- the serial per-group stages on the pair backend with one group
// per lane pair (32 per wave): the throughput build for large group counts (lsg_serial.h).
#define LSG_PAIR_WIDE 1
#include "lsg_serial_pair.hip"
