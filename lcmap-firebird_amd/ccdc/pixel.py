"""ccdc.pixel -- per-pixel processing-mask projection (mirror of reference ccdc/pixel.py)."""
from ccdc._types import ArrayType, ByteType, IntegerType, StructField, StructType, require_pyspark


def table():
    """Cassandra table name"""
    return 'pixel'


def schema():
    """Schema for pixel dataframe"""
    return StructType([
        StructField('cx', IntegerType(), nullable=False),
        StructField('cy', IntegerType(), nullable=False),
        StructField('px', IntegerType(), nullable=False),
        StructField('py', IntegerType(), nullable=False),
        StructField('mask', ArrayType(ByteType()), nullable=True)])


def dataframe(ctx, ccd):
    return ccd.select(schema().fieldNames())


def read(ctx, ids):
    require_pyspark('ccdc.pixel.read (Cassandra storage is out of scope)')


def write(ctx, df):
    require_pyspark('ccdc.pixel.write (Cassandra storage is out of scope)')
