/* compatibility path: reference layout bpe/inc/bpe.h */
#include "../../bpe.h"
