/*
 * PacketTransformer drop-in for SRTPTransformer (transform/srtp/
 * SRTPTransformer.java:70-219) on the MI355X engine.  Swap-in points:
 * tf/sdes/SDesTransformEngine.java:79-97, tf/dtls/DtlsPacketTransformer.java
 * :694-707.  NOT COMPILED IN THIS REPOSITORY (no JDK); see INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

import java.util.function.*;

import org.jitsi.impl.neomedia.*;
import org.jitsi.impl.neomedia.transform.*;

public class GpuSRTPTransformer
    implements PacketTransformer
{
    static final int KIND_RTP = 0, KIND_RTCP = 1;

    final int tid;
    private final Predicate<RawPacket> packetPredicate;
    private int exceptionsInTransform, exceptionsInReverseTransform;

    public GpuSRTPTransformer(GpuSRTPContextFactory forward, GpuSRTPContextFactory reverse)
    {
        this(KIND_RTP, forward, reverse, null);
    }

    GpuSRTPTransformer(int kind, GpuSRTPContextFactory forward, GpuSRTPContextFactory reverse,
                       Predicate<RawPacket> packetPredicate)
    {
        this.packetPredicate = packetPredicate;
        tid = SrtpMi355x.check(SrtpMi355x.transformerCreate(SrtpMi355x.dispatch(), kind, forward.id,
                                                            reverse.id));
    }

    /** SRTPTransformer.setContextFactory: contexts survive (SDES rekey). */
    public void setContextFactory(GpuSRTPContextFactory factory, boolean forward)
    {
        SrtpMi355x.check(SrtpMi355x.transformerSetFactory(SrtpMi355x.dispatch(), tid, factory.id, forward));
    }

    @Override
    public void close()
    {
        SrtpMi355x.transformerClose(SrtpMi355x.dispatch(), tid);
    }

    @Override
    public RawPacket[] transform(RawPacket[] pkts)
    {
        return run(pkts, false);
    }

    @Override
    public RawPacket[] reverseTransform(RawPacket[] pkts)
    {
        return run(pkts, true);
    }

    /** SinglePacketTransformer.java:121-216 over the whole array at once. */
    private RawPacket[] run(RawPacket[] pkts, boolean reverse)
    {
        if (pkts == null || pkts.length == 0)
            return pkts;
        int[] skip = null;
        if (packetPredicate != null)
        {
            skip = new int[pkts.length];
            for (int i = 0; i < pkts.length; i++)
                if (pkts[i] != null && !packetPredicate.test(pkts[i]))
                    skip[i] = 1;
        }
        int r = SrtpMi355x.check(SrtpMi355x.transformPackets(SrtpMi355x.batch(), reverse, tid, pkts, skip));
        if (r > 0)
        {
            if (reverse)
                exceptionsInReverseTransform++;
            else
                exceptionsInTransform++;
            throw new RuntimeException("Failed to " + (reverse ? "reverse-" : "")
                                       + "transform RawPacket(s)! (element " + (r - 1) + ")");
        }
        return pkts;
    }
}
