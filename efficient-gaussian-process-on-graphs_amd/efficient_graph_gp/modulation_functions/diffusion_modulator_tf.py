"""TensorFlow diffusion modulator (reference diffusion_modulator_tf.py:3-9); needs tensorflow."""
import tensorflow as tf  # noqa: F401  (ImportError when absent, as in the reference)


def diffusion_modulator_tf(length, beta):
    length = tf.cast(length, tf.float64)
    beta = tf.cast(beta, tf.float64)
    return tf.pow(-beta, length) / (tf.pow(tf.constant(2.0, tf.float64), length) * tf.exp(tf.math.lgamma(length + 1.0)))
