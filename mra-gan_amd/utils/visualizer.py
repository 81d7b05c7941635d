"""Loss logging (reference utils/visualizer.py:6-27): same line format on stdout and in
<checkpoints_dir>/<name>/loss_log.txt."""
import os
import time


class Visualizer():
    def __init__(self, opt):
        self.name = opt.name
        self.opt = opt
        self.saved = False
        self.log_name = os.path.join(opt.checkpoints_dir, opt.name, 'loss_log.txt')
        os.makedirs(os.path.dirname(self.log_name), exist_ok=True)
        with open(self.log_name, "a") as log_file:
            log_file.write('================ Training Loss (%s) ================\n' % time.strftime("%c"))

    def reset(self):
        self.saved = False

    def print_current_losses(self, epoch, i, losses, t, t_data):
        message = '(epoch: %d, iters: %d, time: %.3f, data: %.3f) ' % (epoch, i, t, t_data)
        message += ''.join('%s: %.3f ' % (k, v) for k, v in losses.items())
        print(message)
        with open(self.log_name, "a") as log_file:
            log_file.write('%s\n' % message)
