"""Diagnostic: train.main plumbing, the learning rate / EMA decay each step hands the update."""
import sys, tempfile
sys.path[:0] = ['.', 'iv2019-boosting-semantic-segmentation-with-weak-labels_amd']
import seg_hip
orig = seg_hip.SegContext.apply_update
def traced(self, lr, momentum=0.9, ema_decay_eff=0.0, grad_scale=1.0, stream=None):
    print('apply_update lr', lr, 'momentum', momentum, 'ema', ema_decay_eff, 'scale', grad_scale)
    return orig(self, lr, momentum, ema_decay_eff, grad_scale, stream)
seg_hip.SegContext.apply_update = traced
import train
tmp = tempfile.mkdtemp()
train.main([tmp + "/logs", "cityscapes", "--max_steps", "3", "--compute_dtype", "fp32",
            "--height_feature_extractor", "64", "--width_feature_extractor", "128",
            "--Nb_per_pixel", "2", "--Nb_per_bbox", "0", "--Nb_per_image", "0",
            "--Ntrain", "2", "--Ne", "3", "--learning_rate_boundaries", "1", "2", "3",
            "--learning_rate_initial", "1e-5", "--save_summaries_steps", "1"])
