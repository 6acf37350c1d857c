// lsg_serial_wide.hip -- the serial per-group stages with one item per 16-lane row (four
// items per wave): the build for large group counts (lsg_serial.h, LSG_ROW_WIDE_MIN).
#define LSG_ROWS_PER_ITEM 1
#include "lsg_serial.hip"
