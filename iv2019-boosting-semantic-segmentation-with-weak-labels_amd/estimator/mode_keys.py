"""tf.estimator.ModeKeys string values (the reference compares ``mode`` against these)."""


class ModeKeys(object):
    TRAIN = 'train'
    EVAL = 'eval'
    PREDICT = 'infer'
