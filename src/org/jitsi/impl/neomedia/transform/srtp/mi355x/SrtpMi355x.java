/*
 * Native declarations of the JNI shim src/native/srtp_mi355x/SrtpMi355x.c
 * over the MI355X SRTP engine (include/srtp_mi355x.h), and the process-wide
 * engine state.  The Java classes are not compiled in this repository (no JDK
 * in the build image); the shim is (tests/jni_stub/), see INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

import org.jitsi.impl.neomedia.*;
import org.jitsi.impl.neomedia.transform.srtp.*;
import org.jitsi.service.configuration.*;
import org.jitsi.service.libjitsi.*;
import org.jitsi.util.*;

public final class SrtpMi355x
{
    static
    {
        // src/org/jitsi/util/JNIUtils.java:37-66, as libjnopenssl is loaded
        JNIUtils.loadLibrary("jnsrtp_mi355x", SrtpMi355x.class.getClassLoader());
    }

    /**
     * The number of GPUs to shard over (default: every device the HIP runtime
     * reports, srtp_device_count).
     */
    public static final String GPUS_PNAME = "org.jitsi.impl.neomedia.transform.srtp.mi355x.GPUS";

    /**
     * The per-packet aggregator's lanes (one per GPU): packets and megabytes
     * per bundle, and pinned bundle slots.  The pinned-memory budget is
     * SLOTS x MB per GPU, on the host and on the device; the defaults (16384,
     * 24, 8: 192 MB per GPU) are where the queued path measured fastest, and
     * 0 or a negative value keeps a default.
     */
    public static final String LANE_PACKETS_PNAME = "org.jitsi.impl.neomedia.transform.srtp.mi355x.LANE_PACKETS";
    public static final String LANE_MB_PNAME = "org.jitsi.impl.neomedia.transform.srtp.mi355x.LANE_MB";
    public static final String LANE_SLOTS_PNAME = "org.jitsi.impl.neomedia.transform.srtp.mi355x.LANE_SLOTS";

    /** One dispatcher per process: every GPU of the node, SSRC-sharded. */
    private static long dispatch;

    /**
     * One aggregator per process over it: the per-packet calls' bundles.
     * Read on every per-packet call, so it is published once (volatile) and
     * read without a lock.
     */
    private static volatile long aggregator;

    public static synchronized long dispatch()
    {
        if (dispatch == 0)
        {
            // SRTPCryptoContext.readConfigurationServicePropertiesOnce
            // (SRTPCryptoContext.java:105-121): the same property, the same default
            boolean checkReplay = true;
            int n = deviceCount();
            ConfigurationService cfg = LibJitsi.getConfigurationService();
            if (cfg != null)
            {
                checkReplay = cfg.getBoolean(SRTPCryptoContext.CHECK_REPLAY_PNAME, checkReplay);
                n = cfg.getInt(GPUS_PNAME, n);
            }
            if (n < 1)
                throw new IllegalStateException("srtp_mi355x: no GPU");
            int[] devices = new int[n];
            for (int i = 0; i < n; i++)
                devices[i] = i;
            dispatch = dispatchCreate(devices, checkReplay, 0);
            if (dispatch == 0)
                throw new IllegalStateException("srtp_mi355x: no engine");
        }
        return dispatch;
    }

    static long aggregator()
    {
        long a = aggregator;
        if (a != 0)
            return a;
        synchronized (SrtpMi355x.class)
        {
            if (aggregator == 0)
            {
                int packets = 0, mb = 0, slots = 0;
                ConfigurationService cfg = LibJitsi.getConfigurationService();
                if (cfg != null)
                {
                    packets = cfg.getInt(LANE_PACKETS_PNAME, packets);
                    mb = cfg.getInt(LANE_MB_PNAME, mb);
                    slots = cfg.getInt(LANE_SLOTS_PNAME, slots);
                }
                a = aggregatorCreate(dispatch(), packets, mb, slots);
                if (a == 0)
                    throw new IllegalStateException("srtp_mi355x: no aggregator");
                aggregator = a;
            }
            return aggregator;
        }
    }

    static int check(int rc)
    {
        if (rc < 0)
            throw new RuntimeException("srtp_mi355x error " + rc);
        return rc;
    }

    static native int deviceCount();
    static native long dispatchCreate(int[] devices, boolean checkReplay, int maxContexts);
    static native void dispatchDestroy(long d);
    static native int factoryCreate(long d, boolean sender, byte[] key, byte[] salt, int[] srtpPolicy,
                                    int[] srtcpPolicy);
    static native int factoryClose(long d, int factory);
    static native int transformerCreate(long d, int kind, int fwd, int rev);
    static native int transformerSetFactory(long d, int transformer, int factory, boolean forward);
    static native int transformerClose(long d, int transformer);
    /**
     * 0, 1 + the first throwing element, or a negative error code.  The
     * calling thread's staging is kept natively and freed when the thread
     * exits; arrays that cannot throw share the aggregator's bundles.
     */
    static native int transformPackets(long d, long aggregator, boolean reverse, int transformer,
                                       RawPacket[] pkts, int[] skip);
    /**
     * srtp_aggregator_create_dispatch with SRTP_AGG_SEAL_IDLE and no callback;
     * lane sizing as the LANE_*_PNAME properties (<= 0: the defaults).
     */
    static native long aggregatorCreate(long d, int maxPackets, int maxMegabytes, int slots);
    static native void aggregatorDestroy(long a);
    /** One packet (srtp_rawpacket_transform_one): its SRTP_STATUS_*, or a negative error code. */
    static native int transformOne(long aggregator, boolean reverse, int transformer, RawPacket pkt);

    /* GpuPacketQueue: srtp_queue_* / srtp_rawpacket_submit / srtp_rawpacket_complete */
    static final int EAGAIN = -6;
    static native long queueCreate(long aggregator, int maxInFlight);
    static native void queueDestroy(long q);
    /** 0, EAGAIN (reap first) or a negative error code. */
    static native int queueSubmit(long q, boolean reverse, int transformer, RawPacket pkt, boolean skip,
                                  long cookie);
    /**
     * Completions in submission order, written back into ring[cookie % ring.length];
     * their statuses in status; the count or a negative error code.
     */
    static native int queueReap(long q, RawPacket[] ring, int[] status, boolean wait);
}
