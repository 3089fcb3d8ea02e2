/*
 * Native declarations of the JNI shim src/native/srtp_mi355x/SrtpMi355x.c
 * over the MI355X SRTP engine (include/srtp_mi355x.h).  NOT COMPILED IN THIS
 * REPOSITORY (no JDK in the build image); see INTEGRATION.md.
 */
package org.jitsi.impl.neomedia.transform.srtp.mi355x;

import org.jitsi.impl.neomedia.*;
import org.jitsi.util.*;

public final class SrtpMi355x
{
    static
    {
        // src/org/jitsi/util/JNIUtils.java:37-66, as libjnopenssl is loaded
        JNIUtils.loadLibrary("jnsrtp_mi355x", SrtpMi355x.class.getClassLoader());
    }

    /** One dispatcher per process: every GPU of the node, SSRC-sharded. */
    private static long dispatch;

    private static final ThreadLocal<Long> BATCH = new ThreadLocal<>();

    public static synchronized long dispatch()
    {
        if (dispatch == 0)
        {
            int n = Integer.getInteger("org.jitsi.srtp.mi355x.GPUS", 8);
            int[] devices = new int[n];
            for (int i = 0; i < n; i++)
                devices[i] = i;
            dispatch = dispatchCreate(devices, true, 0);
            if (dispatch == 0)
                throw new IllegalStateException("srtp_mi355x: no engine");
        }
        return dispatch;
    }

    /** The calling thread's RawPacket[] staging (srtp_rawpacket_batch). */
    static long batch()
    {
        Long b = BATCH.get();
        if (b == null)
        {
            b = batchCreate(dispatch());
            BATCH.set(b);
        }
        return b;
    }

    static int check(int rc)
    {
        if (rc < 0)
            throw new RuntimeException("srtp_mi355x error " + rc);
        return rc;
    }

    static native long dispatchCreate(int[] devices, boolean checkReplay, int maxContexts);
    static native void dispatchDestroy(long d);
    static native int factoryCreate(long d, boolean sender, byte[] key, byte[] salt, int[] srtpPolicy,
                                    int[] srtcpPolicy);
    static native int factoryClose(long d, int factory);
    static native int transformerCreate(long d, int kind, int fwd, int rev);
    static native int transformerSetFactory(long d, int transformer, int factory, boolean forward);
    static native int transformerClose(long d, int transformer);
    static native long batchCreate(long d);
    static native void batchDestroy(long b);
    /** 0, 1 + the first throwing element, or a negative error code. */
    static native int transformPackets(long batch, boolean reverse, int transformer, RawPacket[] pkts,
                                       int[] skip);
}
