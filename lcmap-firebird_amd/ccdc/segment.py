"""ccdc.segment -- segment output schema and projection (mirror of reference ccdc/segment.py).

``read`` / ``write`` go to Cassandra in the reference (segment.py:73-100, cassandra.py); that
storage layer is out of scope and raises here unless pyspark and the
connector are provided by the deployment."""
from ccdc._types import ArrayType, FloatType, IntegerType, StringType, StructField, StructType, require_pyspark


def table():
    """ Cassandra segment table name """
    return 'segment'


def schema():
    return StructType([
        StructField('cx', IntegerType(), nullable=False),
        StructField('cy', IntegerType(), nullable=False),
        StructField('px', IntegerType(), nullable=False),
        StructField('py', IntegerType(), nullable=False),
        StructField('sday', StringType(), nullable=False),
        StructField('eday', StringType(), nullable=False),
        StructField('bday', StringType(), nullable=True),
        StructField('chprob', FloatType(), nullable=True),
        StructField('curqa', IntegerType(), nullable=True),
        StructField('blmag', FloatType(), nullable=True),
        StructField('grmag', FloatType(), nullable=True),
        StructField('remag', FloatType(), nullable=True),
        StructField('nimag', FloatType(), nullable=True),
        StructField('s1mag', FloatType(), nullable=True),
        StructField('s2mag', FloatType(), nullable=True),
        StructField('thmag', FloatType(), nullable=True),
        StructField('blrmse', FloatType(), nullable=True),
        StructField('grrmse', FloatType(), nullable=True),
        StructField('rermse', FloatType(), nullable=True),
        StructField('nirmse', FloatType(), nullable=True),
        StructField('s1rmse', FloatType(), nullable=True),
        StructField('s2rmse', FloatType(), nullable=True),
        StructField('thrmse', FloatType(), nullable=True),
        StructField('blcoef', ArrayType(FloatType()), nullable=True),
        StructField('grcoef', ArrayType(FloatType()), nullable=True),
        StructField('recoef', ArrayType(FloatType()), nullable=True),
        StructField('nicoef', ArrayType(FloatType()), nullable=True),
        StructField('s1coef', ArrayType(FloatType()), nullable=True),
        StructField('s2coef', ArrayType(FloatType()), nullable=True),
        StructField('thcoef', ArrayType(FloatType()), nullable=True),
        StructField('blint', FloatType(), nullable=True),
        StructField('grint', FloatType(), nullable=True),
        StructField('reint', FloatType(), nullable=True),
        StructField('niint', FloatType(), nullable=True),
        StructField('s1int', FloatType(), nullable=True),
        StructField('s2int', FloatType(), nullable=True),
        StructField('thint', FloatType(), nullable=True),
        StructField('rfrawp', ArrayType(FloatType()), nullable=True),
    ])


def dataframe(ctx, ccd):
    """Segment projection of the ccd dataframe (segment.py:59-70)."""
    return ccd.select(schema().fieldNames())


def rows(ccd_rows):
    """Segment projection of format() row dicts (the dataframe() projection without Spark)."""
    names = schema().fieldNames()
    return [{k: r.get(k) for k in names} for r in ccd_rows]


def read(ctx, ids):
    require_pyspark('ccdc.segment.read (Cassandra storage is out of scope)')


def write(ctx, df):
    require_pyspark('ccdc.segment.write (Cassandra storage is out of scope)')


def join(segments, predictions):
    """Join segments dataframe with predictions dataframe (segment.py:103-116)."""
    return segments.join(predictions, on=['cx', 'cy', 'px', 'py', 'sday', 'eday'],
                         how='inner').drop(segments['rfrawp'])
