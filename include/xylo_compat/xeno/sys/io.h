// xeno/sys/io.h (xylo-hip drop-in layer).  ppo2_training.cc includes it but
// uses nothing from it; the weights writer of the path is
// xylo::save_parameters (xylo/nn.h), which writes the same raw float layout
// deep_agent.cc maps.
#ifndef XYLO_HIP_COMPAT_XENO_SYS_IO_H_
#define XYLO_HIP_COMPAT_XENO_SYS_IO_H_
#include <xeno/sys/file_descriptor.h>
#endif  // XYLO_HIP_COMPAT_XENO_SYS_IO_H_
